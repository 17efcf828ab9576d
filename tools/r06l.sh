set -o pipefail
mkdir -p gpurun_out
ok() { rc=$?; [ $rc -le 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ce3.py tests/test_gpu_stage_ops.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06l_tests.log 2>&1; ok &&
timeout -k 10 900 python -u tools/bench_ab.py c2dsr_amd.losshead.CE_LOGITS 3 > gpurun_out/r06l_ab.log 2>&1
