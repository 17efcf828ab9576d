#!/bin/bash
# bf16-output attention backward with a scalar wave index: micro, tests, bf16-line and fp32-line A/B vs previous build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default prev; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -2 || exit 1
done
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 150 -k "attn or module_api or bf16 or stage_ops" > gpurun_out/ob_test.log 2>&1; tail -1 gpurun_out/ob_test.log
bash tools/lib_ab.sh 2 default prev -- --precision bf16
bash tools/lib_ab.sh 1 default prev
