#!/bin/bash
# One GPU cycle on the MI355X box: GPU tests, a bench line, a rocprofv3 kernel-stats profile.
# usage: bash tools/gpu_cycle.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -m pytest tests -m gpu -x -q "${KA[@]}" > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$TAG 6 30
