#!/bin/bash
# split-partial sums with four loads in flight: wgemm tests, wg timing old vs new
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp27.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py tests/test_gpu_kernels.py -q -x -k "wgemm or wg_" --timeout 200 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
for r in 1 2; do for v in old new; do L=c2dsr_amd/libc2dsr_hip.so; [ $v = old ] && L=variants/lib_old.so
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py wg 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O || exit 1; done; done
grep -E "passed|failed|x3 dY" $O
