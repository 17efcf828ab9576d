#!/bin/bash
# K5 at two waves per SIMD (variants/lib_ce8.so: CE3_NW = CE3B_NW = 8) against the default: ce3 micro at MB head-b
# shapes, then the ce3 tests on the variant
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp8.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for v in base ce8 ce8p; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L run python -u tools/ce3_micro.py || { cat $O; exit 1; }
  C2DSR_LIB=$L run python -u tools/ce3_micro.py 18944 36845 || { cat $O; exit 1; }; done
C2DSR_LIB=variants/lib_ce8.so run python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread
cat $O
