#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, no other tracing):
#   FETCH_SIZE | WRITE_SIZE | SQ stall/issue breakdown.  usage: bash tools/pmc.sh TAG [python args]
#   (default args: a short bench.py run)
set -o pipefail
TAG=${1:-pmc}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p gpurun_out
shift
ARGS=${*:-bench.py --steps 2 --warmup 1 --no-cpu-baseline}
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- python3 $ARGS > gpurun_out/${TAG}_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- python3 $ARGS > gpurun_out/${TAG}_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/${TAG}_sq -o run --output-format csv -- python3 $ARGS > gpurun_out/${TAG}_sq.log 2>&1
rc=$?
ls -R gpurun_out/${TAG}_fetch | head
exit $rc
