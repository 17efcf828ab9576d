#!/bin/bash
# Quick GPU check: the GPU suite (optionally -k EXPR) and one bench line (no CPU baseline / extras unless asked).
#   usage: bash tools/quick.sh TAG [pytest -k expr] [bench args...]
set -o pipefail
TAG=${1:-q}
K=${2:-}
shift $(( $# < 2 ? $# : 2 ))
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${KA[@]}" > gpurun_out/${TAG}_gputest.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_gputest.log
[ $rc -eq 0 ] || { grep -E "Error|error|FAILED|assert" gpurun_out/${TAG}_gputest.log | head -30; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
