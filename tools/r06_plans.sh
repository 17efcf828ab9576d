#!/bin/bash
# Batched index plans: their tests, a same-box A/B of the main line (batched vs plan by plan), a kernel trace.
set -o pipefail
TAG=${1:-r06pl}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_index_errors.py tests/test_gpu_stage_ops.py tests/test_gpu_torch_ops.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 700 python tools/bench_ab.py c2dsr_amd.ops.PLANS_BATCHED 3 > gpurun_out/${TAG}_ab.log 2>&1 || { tail -30 gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof 13 40 > gpurun_out/${TAG}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_gaps.txt 2>&1
head -30 gpurun_out/${TAG}_summary.txt
