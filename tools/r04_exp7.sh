#!/bin/bash
# rg3 projection kernel at 8 waves per workgroup (variants/lib_rg8.so) against the default: micro + its tests
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp7.log
: > $O
for v in base rg8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py x3 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }; done
C2DSR_LIB=variants/lib_rg8.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k rgemm --timeout 200 --timeout-method thread >> $O 2>&1
cat $O
