#!/bin/bash
# Eager per-table GCN backward: its test, the DP / parity tests it touches, a same-box A/B of the main line.
set -o pipefail
TAG=${1:-r06eg}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_eager_gcn.py tests/test_gpu_rccl.py tests/test_gpu_dropin_dp.py tests/test_gpu_parity.py tests/test_gpu_stage_ops.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 500 python tools/bench_ab.py c2dsr_amd.ops.EAGER_GCN 2 > gpurun_out/${TAG}_ab.log 2>&1 || { tail -30 gpurun_out/${TAG}_ab.log; exit 1; }
cat gpurun_out/${TAG}_ab.log
