#!/bin/bash
# fused embedding backward: correctness (kernel test) + micro timing; K5 / wg variants
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp5.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
run ./tools/peak/s_phase 20000
run python -u -m pytest tests/test_gpu_kernels.py -q -x -k embed --timeout 200 --timeout-method thread || { cat $O; exit 1; }
run python -u tools/embed_micro.py || { cat $O; exit 1; }
for v in base bivn5 bivn8 bivn5ds3 bivn5dt3; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O; C2DSR_LIB=$L run python -u tools/ce3_micro.py || exit 1; done
for v in base wg8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O; C2DSR_LIB=$L run python -u tools/rg_micro.py wg || exit 1; done
C2DSR_LIB=variants/lib_wg8.so run python -u -m pytest tests/test_gpu_ce3.py -q -x -k wgemm --timeout 200 --timeout-method thread
cat $O
