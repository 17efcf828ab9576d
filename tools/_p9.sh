#!/bin/bash
# attention descriptor variants: micro + same-box step A/B (default / srsrc / attn_old) + attention tests on srsrc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default srsrc attn_old; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -1 || exit 1
done > gpurun_out/srsrc_micro.log
cat gpurun_out/srsrc_micro.log | cut -c1-200
timeout -k 10 200 env C2DSR_LIB_DIR=variants/srsrc python3 -u -m pytest tests -m gpu -q --timeout 100 -k "attn or module_api" > gpurun_out/srsrc_test.log 2>&1; tail -1 gpurun_out/srsrc_test.log
bash tools/lib_ab.sh 2 default srsrc attn_old
