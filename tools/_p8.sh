#!/bin/bash
# kernel stats of the default bench line for two library builds (default vs variants/attn_old)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default attn_old; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  rm -rf gpurun_out/pv_$v
  timeout -k 10 300 env C2DSR_LIB_DIR=$D rocprofv3 --kernel-trace --stats -d gpurun_out/pv_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --steps 5 --warmup 2 > gpurun_out/pv_$v.log 2>&1 || exit 1
  python tools/prof_summary.py gpurun_out/pv_$v 8 40 > gpurun_out/pv_${v}_summary.txt 2>&1
done
head -22 gpurun_out/pv_default_summary.txt | cut -c1-120
head -22 gpurun_out/pv_attn_old_summary.txt | cut -c1-120
