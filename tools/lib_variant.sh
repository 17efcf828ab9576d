#!/bin/bash
# a variant build of the kernel library with one source file rebuilt (current tree, extra flags), next to a copy of
# the operator library (which loads the kernel library from its own directory):
#   bash tools/lib_variant.sh NAME SOURCE.hip "FLAGS" [REPLACES]  -> variants/NAME/{libc2dsr_hip.so, libc2dsr_torch.so}
#   (the other objects from build/; REPLACES = the build/ object the source stands in for, default its base name)
#   use: C2DSR_LIB_DIR=variants/NAME python ...
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
base=$(basename "$src" .hip)
repl=${4:-$base}
mkdir -p variants/$name build/var_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result $flags -c "$src" \
  -o build/var_$name/$base.o
objs=$(ls build/*.o | grep -v "/$repl.o$" | grep -v "/torch_")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$name/$base.o -o variants/$name/libc2dsr_hip.so
cp c2dsr_amd/libc2dsr_torch.so variants/$name/
echo "variants/$name ($src $flags)"
