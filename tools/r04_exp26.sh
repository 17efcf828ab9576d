#!/bin/bash
# GradSink prefill on the side stream: parity + module tests, then a same-box bench A/B of the switch
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp26.log
: > $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_module_api.py -q -x --timeout 300 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 1000 python -u tools/bench_ab.py c2dsr_amd.ops.GRADSINK_PREFILL 3 >> $O 2>&1
grep -E "passed|failed|seq/s" $O
