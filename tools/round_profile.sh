#!/bin/bash
# Round evidence on the MI355X box: the default bench line (with the CPU baseline), a rocprofv3
# --kernel-trace --stats profile of the headline line (no extra lines), and separate FETCH_SIZE / WRITE_SIZE PMC passes.
# usage: bash tools/round_profile.sh TAG      (outputs under gpurun_out/TAG_*)
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
A="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/${TAG}_sq -o run --output-format csv -- python3 $A > gpurun_out/${TAG}_sq.log 2>&1
