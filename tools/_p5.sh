#!/bin/bash
# one-off: bf16 K5 at two waves per SIMD (CE3B_NW=8) vs default, interleaved; FK and MB head shapes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for v in default b8 b8dq2 b8ds3; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v $rep"
  timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/ce3b_micro.py 9472 34886 0 1 2>&1 | grep ce3b || exit 1
  timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/ce3b_micro.py 18944 63937 0 1 2>&1 | grep ce3b || exit 1
done; done > gpurun_out/b8.log
cut -c1-200 gpurun_out/b8.log
timeout -k 10 120 env C2DSR_LIB_DIR=variants/b8 python3 -u -m pytest tests/test_gpu_ce3.py -m gpu -q --timeout 100 -k "ce3b" > gpurun_out/b8_test.log 2>&1; tail -1 gpurun_out/b8_test.log
