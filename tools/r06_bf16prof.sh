#!/bin/bash
# Kernel traces of the bf16 lines (FK = configs[1], MB) and the host lead of the fp32 main line.
set -o pipefail
TAG=${1:-r06bf}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in fk mb; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}${c}_prof -o run --output-format csv -- python3 bench.py --config $c --precision bf16 --no-cpu-baseline --no-extra > gpurun_out/${TAG}${c}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}${c}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}${c}_prof 13 40 > gpurun_out/${TAG}${c}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}${c}_prof > gpurun_out/${TAG}${c}_gaps.txt 2>&1
tail -1 gpurun_out/${TAG}${c}_prof.log | cut -c1-200
done
bash tools/r06_lag.sh ${TAG}lag > /dev/null 2>&1 || { echo lag failed; exit 1; }
head -25 gpurun_out/${TAG}lag_lag.txt
