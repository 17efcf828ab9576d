#!/bin/bash
# linear1 forward precision emulations against the C2 / d256 reference steps (tools/linear1_emu.py)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp13.log
: > $O
for m in f64 x6 x3; do echo "== $m" >> $O
  timeout -k 10 300 python -u tools/linear1_emu.py $m 2>&1 | grep -E "worst|passed|failed|AssertionError: \(" >> $O; done
cat $O
