#!/bin/bash
# a variant kernel library with one source file rebuilt (current tree, extra flags):
#   bash tools/lib_variant.sh NAME SOURCE.hip "FLAGS" [REPLACES]  -> variants/lib_NAME.so (the other objects
#   from build/; REPLACES = the build/ object the source stands in for, default its own base name)
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
base=$(basename "$src" .hip)
repl=${4:-$base}
mkdir -p variants build/var_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Iinclude -Wno-unused-result $flags -c "$src" \
  -o build/var_$name/$base.o
objs=$(ls build/*.o | grep -v "/$repl.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs build/var_$name/$base.o -o variants/lib_$name.so
echo "variants/lib_$name.so ($src $flags)"
