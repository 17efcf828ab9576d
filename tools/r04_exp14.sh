#!/bin/bash
# guarded split linear1 with the branch-light epilogue: tests, timing
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp14.log
: > $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x -k "guard or rgemm" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 120 python -u tools/guard_micro.py >> $O 2>&1 || { cat $O; exit 1; }
cat $O
