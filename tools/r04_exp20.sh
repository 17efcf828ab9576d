#!/bin/bash
# classifier weight images cached per weight update: parity suites + loss-head tests, then the bench line
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp20.log
: > $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_module_api.py -q -x --timeout 300 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 420 python3 bench.py --no-cpu-baseline --no-extra >> $O 2>&1 || { tail -20 $O; exit 1; }
grep -E "passed|failed" $O; tail -1 $O | cut -c1-200
