#!/bin/bash
# K5 with the second-product phase on compiler-visible MFMAs in both roles (variants/lib_biu.so) vs the default,
# interleaved A/B at MB head-b shapes, then the ce3 tests on the variant
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp16.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for r in 1 2 3; do for v in base biu; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L run python -u tools/ce3_micro.py || { cat $O; exit 1; }; done; done
C2DSR_LIB=variants/lib_biu.so run python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread
cat $O
