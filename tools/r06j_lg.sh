set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06k_ce3.log 2>&1
KINDS=1,sk,-8 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06k_lg.log 2>&1
C2DSR_LIB_DIR=variants/lge KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06k_lge.log 2>&1
C2DSR_LIB_DIR=variants/lge timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -x -q --timeout 120 --timeout-method thread -k "True or layout" > gpurun_out/r06k_ce3_lge.log 2>&1
