#!/bin/bash
# split-bf16 row attention (re-applied): kernel tests, then the fp32 parity suites against the oracle / reference
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp18.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "attention" --timeout 200 --timeout-method thread >> $O 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread >> $O 2>&1
grep -E "passed|failed|FAILED|Error" $O | tail -20
