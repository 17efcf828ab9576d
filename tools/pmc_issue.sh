#!/bin/bash
# Issue / stall counters (own rocprofv3 passes, no other tracing).  usage: bash tools/pmc_issue.sh TAG
set -o pipefail
TAG=${1:-iss}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS=${ARGS:-"bench.py --steps 2 --warmup 1 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_a -o run --output-format csv -- python3 $ARGS > gpurun_out/${TAG}_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/${TAG}_b -o run --output-format csv -- python3 $ARGS > gpurun_out/${TAG}_b.log 2>&1
