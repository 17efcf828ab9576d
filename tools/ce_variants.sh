#!/bin/bash
# Builds variant kernel libraries with the ce.hip tuning knobs into variants/ (git-ignored .so files that
# travel to the GPU box), for tools/ce_micro.py:  bash tools/ce_variants.sh NAME "-DCE_FWDU_DS=4 ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p build/var_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result $flags \
    -c c2dsr_amd/csrc/ce.hip -o build/var_$name/ce.o
  objs=$(ls build/*.o | grep -v '/ce.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$name/ce.o -o variants/lib_$name.so
  echo "variants/lib_$name.so ($flags)"
done
