#!/bin/bash
# A rocprofv3 kernel-trace profile of the main bench line (+ per-kernel summary and idle gaps), and optionally the
# bench line itself first.   usage: bash tools/prof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-p}
shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extra "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra "$@" > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof 13 45 > gpurun_out/${TAG}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_gaps.txt 2>&1
head -48 gpurun_out/${TAG}_summary.txt
head -12 gpurun_out/${TAG}_gaps.txt
