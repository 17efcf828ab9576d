set -o pipefail
mkdir -p gpurun_out
for v in tiny plain; do
C2DSR_LIB_DIR=variants/$v KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06u_$v.log 2>&1 || exit 1
done
KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06u_def.log 2>&1
