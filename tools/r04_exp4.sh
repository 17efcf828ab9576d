#!/bin/bash
# K5 schedule variants (CE3_BI): head b and head a shapes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp4.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for v in base bivn5 bivn8 bivn5ds3 bivn5dq1 bivn5dt3 base; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O; C2DSR_LIB=$L run python -u tools/ce3_micro.py || exit 1; C2DSR_LIB=$L run python -u tools/ce3_micro.py 18944 36845 || exit 1; done
cat $O
