#!/bin/bash
# guarded linear1 (caller-kept norms, one flag byte per lane): guard tests, micro, reference steps
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp22.log
: > $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py tests/test_gpu_torch_ops.py -q -x -k "guard or rgemm or torch_ops" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 120 python -u tools/guard_micro.py >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "c2_step or d256 or golden" --timeout 300 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
grep -E "passed|failed|linear1 M" $O
