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
