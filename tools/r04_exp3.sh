#!/bin/bash
# K5 on compiler-visible MFMAs (CE3_BI variants): timing, phase stamps, correctness (ce3 tests on the variant)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp3.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for v in base bi bivn2 bivn5; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O; C2DSR_LIB=$L run python -u tools/ce3_micro.py || exit 1; C2DSR_LIB=$L run python -u tools/ce3_micro.py 18944 36845 || exit 1; done
C2DSR_LIB=variants/lib_bistamp.so run python -u tools/ce3_micro.py || exit 1
C2DSR_LIB=variants/lib_bi.so run python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread || exit 1
cat $O
