#!/bin/bash
# Round-6 profiling pass: the main line's kernel trace (+ idle gaps), the C4 per-GPU slice (EE sizes, B = 512) kernel
# trace and host enqueue time.   usage: bash tools/prof_r06.sh TAG
set -o pipefail
TAG=${1:-r06p}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof 13 60 > gpurun_out/${TAG}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_gaps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}ee_prof -o run --output-format csv -- python3 bench.py --config ee --batch 512 --no-cpu-baseline --no-extra > gpurun_out/${TAG}ee_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}ee_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}ee_prof 13 60 > gpurun_out/${TAG}ee_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}ee_prof 12 > gpurun_out/${TAG}ee_gaps.txt 2>&1
timeout -k 10 300 python3 tools/host_time.py fp32 ee 512 60 > gpurun_out/${TAG}ee_host.txt 2>&1 || { tail -20 gpurun_out/${TAG}ee_host.txt; exit 1; }
timeout -k 10 300 python3 tools/host_time.py fp32 mb 0 10 > gpurun_out/${TAG}mb_host.txt 2>&1 || { tail -20 gpurun_out/${TAG}mb_host.txt; exit 1; }
head -3 gpurun_out/${TAG}ee_host.txt; head -3 gpurun_out/${TAG}mb_host.txt
head -12 gpurun_out/${TAG}_summary.txt
