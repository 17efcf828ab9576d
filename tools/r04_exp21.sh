#!/bin/bash
# guarded linear1 with caller-kept norms + vectorised flag scan: guard tests, micro, reference steps; then the A/B of the
# cached classifier weight images on the bench line
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp21.log
: > $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k "guard or rgemm" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 120 python -u tools/guard_micro.py >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "c2_step or d256" --timeout 300 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fk.py -q -s --timeout 300 --timeout-method thread 2>&1 | grep -E "FK \(|passed|failed" >> $O
timeout -k 10 900 python -u tools/bench_ab.py c2dsr_amd.losshead.CACHE_CE_WEIGHTS 2 >> $O 2>&1
grep -E "passed|failed|linear1 M|seq/s|FK \\(" $O | cut -c1-1500
