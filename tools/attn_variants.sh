#!/bin/bash
# variant kernel libraries with attention.hip knobs (see tools/attn_micro.py): NAME "FLAGS" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result $flags \
    -c c2dsr_amd/csrc/attention.hip -o build/var_$name/attention.o
  objs=$(ls build/*.o | grep -v '/attention.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$name/attention.o -o variants/lib_$name.so
  echo "variants/lib_$name.so ($flags)"
done
