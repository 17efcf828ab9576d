#!/bin/bash
# Round evidence, part B (one gpurun call): C5 kernel stats + FETCH / WRITE passes on bf16 tables, FETCH / WRITE passes
# of the C5 fp32-table run, and the GPU suite.   usage: bash tools/evidence_b.sh TAG
set -o pipefail
TAG=${1:-r06z}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="bench.py --config c5 --c5-tables bf16 --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}c5_prof -o run --output-format csv -- python3 $C > gpurun_out/${TAG}c5_prof.log 2>&1 &&
python tools/prof_summary.py gpurun_out/${TAG}c5_prof 3 20 > gpurun_out/${TAG}c5_summary.txt 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}c5_fetch -o run --output-format csv -- python3 $C > gpurun_out/${TAG}c5_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}c5_write -o run --output-format csv -- python3 $C > gpurun_out/${TAG}c5_write.log 2>&1 || { echo "c5 passes failed"; exit 1; }
F="bench.py --config c5 --c5-tables fp32 --steps 2 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}c5f_fetch -o run --output-format csv -- python3 $F > gpurun_out/${TAG}c5f_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}c5f_write -o run --output-format csv -- python3 $F > gpurun_out/${TAG}c5f_write.log 2>&1 || { echo "c5 fp32 passes failed"; exit 1; }
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1; echo "gputest rc=$?"
tail -4 gpurun_out/${TAG}_gputest.log
