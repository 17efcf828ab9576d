set -o pipefail
mkdir -p gpurun_out
for v in nt1 nost nt2; do
C2DSR_LIB_DIR=variants/$v KINDS=1 timeout -k 10 200 python -u tools/ce3_lg_micro.py > gpurun_out/r06o_$v.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C2DSR_LIB_DIR=variants/nt1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/r06o_prof.log 2>&1 &&
python tools/prof_summary.py gpurun_out/r06o_prof 13 40 > gpurun_out/r06o_summary.txt 2>&1
