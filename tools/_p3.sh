#!/bin/bash
# one-off: stream-K dW sweep — ce3 tests, micro A/B (split plan vs stream-K), head-touching step tests, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ce3.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/sk_ce3.log 2>&1; rc=$?
grep -E "errors|passed|failed" gpurun_out/sk_ce3.log | tail -25
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 5 90 python -u tools/ce3_micro.py 18944 63937 0 1 2>&1 | grep "ce3 " || exit 1
  timeout -k 5 90 python -u tools/ce3_micro.py 18944 63937 0 -1 2>&1 | grep "ce3 " || exit 1
  timeout -k 5 90 python -u tools/ce3_micro.py 18944 36845 0 1 2>&1 | grep "ce3 " || exit 1
  timeout -k 5 90 python -u tools/ce3_micro.py 18944 36845 0 -1 2>&1 | grep "ce3 " || exit 1
  timeout -k 5 90 python -u tools/ce3b_micro.py 9472 34886 0 4 2>&1 | grep "ce3b " || exit 1
  timeout -k 5 90 python -u tools/ce3b_micro.py 9472 34886 0 -1 2>&1 | grep "ce3b " || exit 1
  timeout -k 5 90 python -u tools/ce3b_micro.py 9472 29207 0 1 2>&1 | grep "ce3b " || exit 1
  timeout -k 5 90 python -u tools/ce3b_micro.py 9472 29207 0 -1 2>&1 | grep "ce3b " || exit 1
done > gpurun_out/sk_micro.log
cut -c1-250 gpurun_out/sk_micro.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "stage_ops or c2_step or c3_step or fk or loss_head or d256" > gpurun_out/sk_steps.log 2>&1; rc=$?
tail -3 gpurun_out/sk_steps.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/sk_steps.log | head -20; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-c5 > gpurun_out/sk_bench.log 2>&1 || { tail -20 gpurun_out/sk_bench.log; exit 1; }
tail -1 gpurun_out/sk_bench.log | cut -c1-300
