#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp6.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
run ./tools/peak/s_phase 20000 || { cat $O; exit 1; }
run python -u -m pytest tests/test_gpu_kernels.py -q -x -k embed --timeout 200 --timeout-method thread || { cat $O; exit 1; }
run python -u tools/embed_micro.py || { cat $O; exit 1; }
cat $O
O2=gpurun_out/exp6b.log
: > $O2
for v in base rg8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O2; C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py x3 2>&1 | grep -v amdgpu.ids >> $O2 || exit 1; done
C2DSR_LIB=variants/lib_rg8.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k rgemm --timeout 200 --timeout-method thread >> $O2 2>&1
cat $O2
