#!/bin/bash
# Round-6 A/B of the bf16 K5 geometry: 3 stationary blocks × 32-row tiles (default) vs 2 × 64 (variants/b_old), at the
# FK and MB head-b shapes over a few split counts; then the bf16 ce3 float64 tests on the default build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r06_ce3b_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 120 --timeout-method thread >> $out 2>&1 || { tail -30 $out; exit 1; }
for v in "" variants/b_old; do
  for cfg in "9472 34886 3 1" "9472 34886 5 2" "9472 34886 8 4" "18944 63937 5 1" "18944 63937 8 2" "18944 63937 12 1"; do
    C2DSR_LIB_DIR=$v timeout -k 5 60 python -u tools/ce3b_micro.py $cfg 2>&1 | grep ce3b | sed "s|^|${v:-new} |" >> $out || { echo "fail $v $cfg" >> $out; exit 1; }
  done
done
cat $out | tail -14
