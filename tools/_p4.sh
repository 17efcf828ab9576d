#!/bin/bash
# one-off: remainder-split dW plan — ce3 tests, step tests, A/B vs the previous selection, FK line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ce3.py -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/rem_ce3.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/rem_ce3.log | tail -3; grep -E "MB head" gpurun_out/rem_ce3.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/rem_ce3.log | head; exit 1; }
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "stage_ops or c2_step or c3_step or fk or loss_head or d256" > gpurun_out/rem_steps.log 2>&1; rc=$?
tail -1 gpurun_out/rem_steps.log
[ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/rem_steps.log | head -20; exit 1; }
timeout -k 10 800 python3 tools/bench_ab.py c2dsr_amd.losshead.DW_SK 3 > gpurun_out/rem_ab.log 2>&1; tail -2 gpurun_out/rem_ab.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-c5 > gpurun_out/rem_bench.log 2>&1 || { tail -20 gpurun_out/rem_bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/rem_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], {k:(v['value'], v['roofline']['frac']) for k,v in d['extra_lines'].items()})"
