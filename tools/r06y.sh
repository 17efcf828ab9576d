set -o pipefail
mkdir -p gpurun_out
KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py 18944 63937 > gpurun_out/r06y_def.log 2>&1 || exit 1
for v in pat0 dt4 dt3; do
C2DSR_LIB_DIR=variants/$v KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py 18944 63937 > gpurun_out/r06y_$v.log 2>&1 || exit 1
done
