# fp32-mode GPU checks: the fp32 oracle parity at d=256 and a profiled fp32 bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "fp32 or c4" > gpurun_out/fp32_check.log 2>&1; grep -E "PASS|FAIL|passed|failed" gpurun_out/fp32_check.log | tail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fp32_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/fp32_prof.log 2>&1; tail -1 gpurun_out/fp32_prof.log | cut -c1-300
