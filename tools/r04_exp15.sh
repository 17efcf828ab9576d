#!/bin/bash
# guarded split linear1 with k-sequential exact recompute: tests, timing, C2 / d256 reference steps
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp15.log
: > $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k "guard" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 120 python -u tools/guard_micro.py >> $O 2>&1 || { cat $O; exit 1; }
echo "== RELU_GUARD=True" >> $O
timeout -k 10 300 python -u -c "
import sys, pytest
import c2dsr_amd.ops as o
o.RELU_GUARD = True
sys.exit(pytest.main(['tests/test_gpu_parity.py', '-k', 'c2_step or d256_step', '-s', '-q', '-p', 'no:cacheprovider']))
" 2>&1 | grep -E "worst|passed|failed|AssertionError: \(" >> $O
cat $O
