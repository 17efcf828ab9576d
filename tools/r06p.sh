set -o pipefail
mkdir -p gpurun_out
C2DSR_CE_LOGITS_GB=3 timeout -k 10 900 python -u tools/bench_ab.py c2dsr_amd.losshead.CE_LOGITS 3 > gpurun_out/r06p_ab.log 2>&1
