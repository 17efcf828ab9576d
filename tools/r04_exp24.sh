#!/bin/bash
# bf16-mode weight images in fragment order: layout / bit-equality test, the rgemm + parity tests, micro row vs frag,
# then the bf16 bench line
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp24.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py tests/test_gpu_kernels.py -q -x -k "fragment or rgemm or rg_" --timeout 200 --timeout-method thread >> $O 2>&1 || { tail -40 $O; exit 1; }
timeout -k 10 150 python -u tools/rg_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { tail -20 $O; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread >> $O 2>&1 || { tail -40 $O; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra --precision bf16 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -E "passed|failed|b16f? N|seq/s" $O | cut -c1-200; tail -1 $O | cut -c1-200
