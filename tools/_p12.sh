#!/bin/bash
# attention backward with bounded global loads (ATTN_VLD) vs default: micro, tests, fp32-line A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default vld; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -2 || exit 1
done
timeout -k 10 400 env C2DSR_LIB_DIR=variants/vld python3 -u -m pytest tests -m gpu -q --timeout 150 -k "attn or module_api or c2_step or stage_ops or d256" > gpurun_out/vld_test.log 2>&1; tail -1 gpurun_out/vld_test.log
bash tools/lib_ab.sh 2 default vld
