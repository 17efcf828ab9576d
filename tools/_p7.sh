#!/bin/bash
# attention kernels with a scalar wave index (no descriptor waterfall loops): micro, attention/parity tests, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 5 90 python -u tools/attn_micro.py 2>&1 | tail -1 || exit 1
timeout -k 5 90 python -u tools/attn_micro.py 2>&1 | tail -1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "attn or stage_ops or c2_step or c3_step or d256 or dropout or module_api" > gpurun_out/wv_test.log 2>&1; rc=$?
tail -1 gpurun_out/wv_test.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/wv_test.log | head -20; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extra > gpurun_out/wv_bench.log 2>&1 || { tail -20 gpurun_out/wv_bench.log; exit 1; }
tail -1 gpurun_out/wv_bench.log | cut -c1-200
