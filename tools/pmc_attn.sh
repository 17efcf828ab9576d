#!/bin/bash
# TA busy of the attention kernels (fragment-shaped row loads: 32 rows x 32 B per wave instruction)
# vs the projection GEMM (row-contiguous loads), one counter pass on the attention micro-benchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE -d gpurun_out/attn_ta -o run --output-format csv -- python3 tools/attn_micro.py > gpurun_out/attn_ta.log 2>&1 || { tail -20 gpurun_out/attn_ta.log; exit 1; }
python3 - <<'PY'
import csv, glob, re, collections
f = glob.glob('gpurun_out/attn_ta/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name']).split('(')[0]
    acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in acc.items():
    ta = sum(c['TA_BUSY_avr']) / max(1, len(c['TA_BUSY_avr']))
    gui = sum(c['GRBM_GUI_ACTIVE']) / max(1, len(c['GRBM_GUI_ACTIVE'])) / 8
    print(f'{k[:40]:40s} TA_BUSY_avr {ta:12.0f}  GUI cycles/XCD {gui:12.0f}  TA busy frac {ta / gui if gui else 0:.3f}')
PY
