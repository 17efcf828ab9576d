# Builds the gfx950 kernel library (C ABI) in-tree: c2dsr_amd/libc2dsr_hip.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard c2dsr_amd/csrc/*.hip)
OBJ := $(patsubst c2dsr_amd/csrc/%.hip,build/%.o,$(SRC))
HDR := $(wildcard c2dsr_amd/csrc/*.h) include/c2dsr.h
FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result

all: kernels torch

# the kernel library and the host pipeline need no torch; `make kernels` builds them alone
kernels: c2dsr_amd/libc2dsr_hip.so c2dsr_amd/libc2dsr_prep.so
torch: c2dsr_amd/libc2dsr_torch.so

build/%.o: c2dsr_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

c2dsr_amd/libc2dsr_hip.so: $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

# host data pipeline (CPU only, g++)
c2dsr_amd/libc2dsr_prep.so: c2dsr_amd/csrc_host/prep.cpp include/c2dsr_prep.h
	g++ -O3 -fPIC -shared -std=c++17 -Wall -Iinclude $< -o $@

# PyTorch-ROCm extension: TORCH_LIBRARY(c2dsr) over the C ABI (host C++, links the kernel library by rpath)
# (recursively expanded: torch is queried only when the torch target is built, never by `make clean` / `kernels`)
TORCH_DIR ?= $(shell python3 -c 'import os, torch; print(os.path.dirname(torch.__file__))')
TORCH_ABI ?= $(shell python3 -c 'import torch; print(int(torch.compiled_with_cxx11_abi()))')
TORCH_FLAGS = -O2 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=$(TORCH_ABI) \
	-Iinclude -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -I/opt/rocm/include

c2dsr_amd/csrc_torch/torch_ops_gen.inc: include/c2dsr.h tools/gen_torch_ops.py
	python3 tools/gen_torch_ops.py $@

TORCH_SRC := $(wildcard c2dsr_amd/csrc_torch/*.cpp)
TORCH_OBJ := $(patsubst c2dsr_amd/csrc_torch/%.cpp,build/torch_%.o,$(TORCH_SRC))

build/torch_%.o: c2dsr_amd/csrc_torch/%.cpp c2dsr_amd/csrc_torch/c2t.h c2dsr_amd/csrc_torch/torch_ops_gen.inc include/c2dsr.h
	@mkdir -p build
	g++ $(TORCH_FLAGS) -c $< -o $@

c2dsr_amd/libc2dsr_torch.so: $(TORCH_OBJ) c2dsr_amd/libc2dsr_hip.so
	g++ -shared $(TORCH_OBJ) -o $@ -Lc2dsr_amd -lc2dsr_hip -Wl,-rpath,'$$ORIGIN' \
		-L$(TORCH_DIR)/lib -ltorch -ltorch_cpu -lc10 -lc10_hip -ltorch_hip -lamdhip64 -Wl,-rpath,$(TORCH_DIR)/lib

clean:
	rm -rf build c2dsr_amd/libc2dsr_hip.so c2dsr_amd/libc2dsr_prep.so c2dsr_amd/libc2dsr_torch.so

.PHONY: all clean kernels torch
