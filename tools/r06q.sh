set -o pipefail
mkdir -p gpurun_out
C2DSR_PLANS_EARLY=1 timeout -k 10 900 python -u tools/bench_ab.py c2dsr_amd.losshead.CE_LOGITS 3 > gpurun_out/r06q_ab_lg_early.log 2>&1 &&
timeout -k 10 600 python -u tools/bench_ab.py c2dsr_amd.trainer.PLANS_EARLY 2 > gpurun_out/r06q_ab_early.log 2>&1
