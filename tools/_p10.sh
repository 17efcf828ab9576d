#!/bin/bash
# attention backward rows: scalar wave index + the 2x2 path as a call (ATTN_B22) vs default — micro, tests, step A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default b22; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -2 || exit 1
done > gpurun_out/b22_micro.log
cat gpurun_out/b22_micro.log | cut -c1-200
timeout -k 10 300 env C2DSR_LIB_DIR=variants/b22 python3 -u -m pytest tests -m gpu -q --timeout 150 -k "attn or module_api or c2_step or stage_ops" > gpurun_out/b22_test.log 2>&1; tail -1 gpurun_out/b22_test.log
#bash tools/lib_ab.sh 2 default b22
