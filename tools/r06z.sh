set -o pipefail
mkdir -p gpurun_out
ok() { rc=$?; [ $rc -le 1 ]; }
C2DSR_LIB_DIR=variants/g8 timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -x -q --timeout 120 --timeout-method thread -k "True or layout" > gpurun_out/r06z_ce3_g8.log 2>&1; ok &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -x -q --timeout 120 --timeout-method thread -k "True or layout" > gpurun_out/r06z_ce3.log 2>&1; ok &&
KINDS=1,-8 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06z_def.log 2>&1 &&
C2DSR_LIB_DIR=variants/g8 KINDS=1,-8 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06z_g8.log 2>&1
