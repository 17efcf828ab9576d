#!/bin/bash
# GPU cycle: smoke, a bench line, a rocprofv3 kernel-stats profile + idle gaps, then the GPU suite.
#   usage: bash tools/cycle.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof 13 40 > gpurun_out/${TAG}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_gaps.txt 2>&1
head -30 gpurun_out/${TAG}_summary.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1; echo "gputest rc=$?"
tail -15 gpurun_out/${TAG}_gputest.log
