#!/bin/bash
# one-off: K5 second product with single-term bf16 probabilities (CE3_P1 variant) — timing and accuracy
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 120 python3 tools/ce3_micro.py > gpurun_out/p1_micro_def.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 120 env C2DSR_LIB_DIR=variants/p1 python3 tools/ce3_micro.py > gpurun_out/p1_micro_p1.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 300 env C2DSR_LIB_DIR=variants/p1 python3 -u -m pytest tests/test_gpu_ce3.py -m gpu -q -s --timeout 200 --timeout-method thread -k "matches_float64 or rescale" > gpurun_out/p1_ce3.log 2>&1; rc=$?; ok $rc || exit $rc
grep -E "errors|passed|failed" gpurun_out/p1_ce3.log | tail -20
tail -5 gpurun_out/p1_micro_def.log gpurun_out/p1_micro_p1.log
timeout -k 10 120 env C2DSR_LIB_DIR=variants/stamp python3 tools/ce3_micro.py > gpurun_out/stamp_ce3.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 120 env C2DSR_LIB_DIR=variants/stamp python3 tools/ce3b_micro.py > gpurun_out/stamp_ce3b_fk.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 120 env C2DSR_LIB_DIR=variants/stamp python3 tools/ce3b_micro.py 18944 63937 > gpurun_out/stamp_ce3b_mb.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 120 python3 tools/ce3b_micro.py > gpurun_out/ce3b_fk.log 2>&1; rc=$?; ok $rc || exit $rc
cat gpurun_out/stamp_ce3.log gpurun_out/stamp_ce3b_fk.log gpurun_out/stamp_ce3b_mb.log gpurun_out/ce3b_fk.log | cut -c1-300
for ns in 4 5 6 8 12; do timeout -k 5 60 python -u tools/ce3_micro.py 18944 63937 $ns 1 2>&1 | grep "ce3 " || exit 1; done > gpurun_out/fwd_sweep.log
cat gpurun_out/fwd_sweep.log | cut -c1-200
for v in default segu4 segpref segpref4 segch32; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/embed_micro.py 2>&1 | tail -2 || exit 1
done > gpurun_out/embed_var.log
cat gpurun_out/embed_var.log | cut -c1-220
for v in default attnpf attnpf1; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -1 || exit 1
done > gpurun_out/attn_var.log
cat gpurun_out/attn_var.log | cut -c1-250
