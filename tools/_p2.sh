#!/bin/bash
# one-off: K5 built without SLP vectorisation (packed f32 VALU beside MFMAs) vs default, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for v in default noslp; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v $rep"
  timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/ce3b_micro.py 9472 34886 0 4 2>&1 | grep ce3b || exit 1
  timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/ce3b_micro.py 18944 63937 0 1 2>&1 | grep ce3b || exit 1
  timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/ce3_micro.py 18944 63937 0 1 2>&1 | grep "ce3 " || exit 1
done; done > gpurun_out/noslp.log
cut -c1-230 gpurun_out/noslp.log
