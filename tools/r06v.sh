set -o pipefail
mkdir -p gpurun_out
ok() { rc=$?; [ $rc -le 1 ]; }
C2DSR_LIB_DIR=variants/lge2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -x -q --timeout 120 --timeout-method thread -k "True or layout" > gpurun_out/r06v_ce3.log 2>&1; ok &&
for v in lge2 lge2p; do
C2DSR_LIB_DIR=variants/$v KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06v_$v.log 2>&1 || exit 1
done
