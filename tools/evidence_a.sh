#!/bin/bash
# Round evidence, part A (one gpurun call): smoke, the default bench line, rocprofv3 kernel stats of the main line
# (+ idle gaps), FETCH / WRITE / SQ PMC passes of the main line.   usage: bash tools/evidence_a.sh TAG
set -o pipefail
TAG=${1:-r06z}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 480 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof 13 60 > gpurun_out/${TAG}_summary.txt 2>&1
python tools/gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_gaps.txt 2>&1
A="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/${TAG}_sq -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_sq.log 2>&1 || { echo "pmc failed"; exit 1; }
head -25 gpurun_out/${TAG}_summary.txt
