#!/bin/bash
# guarded split linear1 (8 waves, fragment image): its tests, timing against the exact GEMM, and the C2 / d256 reference
# steps' worst errors with the exact linear1 forward vs the guarded split producer
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp12.log
: > $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k "guard or rgemm" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 120 python -u tools/guard_micro.py >> $O 2>&1 || { cat $O; exit 1; }
for g in False True; do echo "== RELU_GUARD=$g" >> $O
  timeout -k 10 300 python -u -c "
import sys, pytest
import c2dsr_amd.ops as o
o.RELU_GUARD = $g
sys.exit(pytest.main(['tests/test_gpu_parity.py', '-k', 'c2_step or d256_step', '-s', '-q', '-p', 'no:cacheprovider']))
" 2>&1 | grep -E "worst|passed|failed|Error|assert" >> $O; done
cat $O
