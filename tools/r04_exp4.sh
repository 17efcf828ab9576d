#!/bin/bash
# K5 schedule variants (CE3_BI): head b and head a shapes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp4.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for v in base bivn5 bivn8 bivn5ds3 bivn5dq1 bivn5dt3 base; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O; C2DSR_LIB=$L run python -u tools/ce3_micro.py || exit 1; C2DSR_LIB=$L run python -u tools/ce3_micro.py 18944 36845 || exit 1; done
cat $O
O2=gpurun_out/exp4b.log
: > $O2
for v in base wg8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O2; C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py wg 2>&1 | grep -v amdgpu.ids >> $O2 || exit 1; done
C2DSR_LIB=variants/lib_wg8.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k wgemm --timeout 200 --timeout-method thread >> $O2 2>&1 || exit 1
cat $O2
