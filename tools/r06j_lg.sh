set -o pipefail
mkdir -p gpurun_out
ok() { rc=$?; [ $rc -le 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ce3.py tests/test_gpu_stage_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06n_ce3.log 2>&1; ok &&
KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06n_lg.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06n_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/r06n_prof.log 2>&1 &&
python tools/prof_summary.py gpurun_out/r06n_prof 13 40 > gpurun_out/r06n_summary.txt 2>&1
