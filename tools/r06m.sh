set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in 1 0; do
C2DSR_CE_LOGITS=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r06m_prof$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/r06m_prof$v.log 2>&1 || exit 1
python tools/prof_summary.py gpurun_out/r06m_prof$v 13 40 > gpurun_out/r06m_summary$v.txt 2>&1
done
