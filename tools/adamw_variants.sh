#!/bin/bash
# variant kernel libraries with adamw.hip knobs (see tools/adamw_micro.py): NAME "FLAGS" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result $flags \
    -c c2dsr_amd/csrc/adamw.hip -o build/var_$name/adamw.o
  objs=$(ls build/*.o | grep -v '/adamw.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$name/adamw.o -o variants/lib_$name.so
  echo "variants/lib_$name.so ($flags)"
done
