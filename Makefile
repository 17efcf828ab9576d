# Builds the gfx950 kernel library (C ABI) in-tree: c2dsr_amd/libc2dsr_hip.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard c2dsr_amd/csrc/*.hip)
OBJ := $(patsubst c2dsr_amd/csrc/%.hip,build/%.o,$(SRC))
HDR := $(wildcard c2dsr_amd/csrc/*.h) include/c2dsr.h
FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result

all: c2dsr_amd/libc2dsr_hip.so c2dsr_amd/libc2dsr_prep.so

build/%.o: c2dsr_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

c2dsr_amd/libc2dsr_hip.so: $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

# host data pipeline (CPU only, g++)
c2dsr_amd/libc2dsr_prep.so: c2dsr_amd/csrc_host/prep.cpp include/c2dsr_prep.h
	g++ -O3 -fPIC -shared -std=c++17 -Wall -Iinclude $< -o $@

clean:
	rm -rf build c2dsr_amd/libc2dsr_hip.so c2dsr_amd/libc2dsr_prep.so

.PHONY: all clean
