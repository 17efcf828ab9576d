set -o pipefail
mkdir -p gpurun_out
ok() { rc=$?; [ $rc -le 1 ]; }
C2DSR_PLANS_EARLY=1 C2DSR_CE_LOGITS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stage_ops.py tests/test_gpu_driver.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06r_tests.log 2>&1; ok &&
timeout -k 10 900 python -u tools/bench_ab.py c2dsr_amd.losshead.CE_LOGITS,c2dsr_amd.trainer.PLANS_EARLY 3 > gpurun_out/r06r_ab.log 2>&1
