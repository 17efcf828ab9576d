set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_ce3.py > gpurun_out/ce3_test.log 2>&1; grep -E "errors|passed|failed" gpurun_out/ce3_test.log | tail -12
timeout -k 10 300 python3 bench.py --precision fp32 --no-cpu-baseline --no-extra > gpurun_out/fp32_bench.log 2>&1; tail -1 gpurun_out/fp32_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp32_prof -o run --output-format csv -- python3 bench.py --precision fp32 --no-cpu-baseline --no-extra > gpurun_out/fp32_prof.log 2>&1
ls gpurun_out/fp32_prof/*/ 2>/dev/null | head
