#!/bin/bash
set -o pipefail
TAG=${1:-r06lag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --steps 4 --warmup 2 > gpurun_out/${TAG}.log 2>&1 || { tail -20 gpurun_out/${TAG}.log; exit 1; }
python tools/host_lag.py gpurun_out/${TAG} > gpurun_out/${TAG}_lag.txt 2>&1
cat gpurun_out/${TAG}_lag.txt
rm -f gpurun_out/${TAG}/*hip_api_trace.csv gpurun_out/${TAG}/*/*hip_api_trace.csv 2>/dev/null; true
