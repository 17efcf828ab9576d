"""K5 HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE passes of tools/round_profile.sh:
FETCH_SIZE (KB) doubled per the gfx950 correction (MI355X_MICROARCH.md §HBM), WRITE_SIZE (KB) as is.
Also the K1 + K2 kernels (GCN SpMM, embedding gather / segment sums) per step → hbm_traffic.json next to
the K5 file (the PMC run is bench.py --steps 2 --warmup 1: 3 steps).
usage: python tools/pmc_traffic.py gpurun_out/TAG [profiles/k5_traffic_fp32.json] [fp32|bf16]
       python tools/pmc_traffic.py gpurun_out/TAG profiles/c5_traffic.json c5   (the C5 line: bench.py --config c5
       --c5-tables bf16 --steps 2 --warmup 1; K1 + K2 only, written to the given file)
(the precision of the profiled bench line selects the K5 kernels: ce3.hip's split (fp32 mode) or plain-bf16
instantiation; the K1+K2
file is written next to the K5 file as hbm_traffic[_fp32].json)"""
import csv
import json
import re
import subprocess
import sys
from collections import defaultdict

pre = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None
prec = sys.argv[3] if len(sys.argv) > 3 else 'fp32'
# the kernels the two timed K5 entry points launch per head (fwd_u: sweep + rows; dw: sweep)
# (ce3_kernel<D, MODE, SPLIT, NW>: SPLIT = true in the fp32 mode, false for the plain-bf16 instantiation; matched
# without the trailing arguments)
K5 = (('ce3_kernel<256, 0, false', 'ce_rows_kernel', 'ce3_kernel<256, 1, false') if prec == 'bf16' else
      ('ce3_kernel<256, 0, true', 'ce_rows_kernel', 'ce3_kernel<256, 1, true', 'ce3_dwl_kernel'))
# (fp32 mode with the logits kept, losshead.CE_LOGITS: the forward is ce3_kernel<256, 0, true, 4, true> — the same
# prefix — and the dW sweep ce3_dwl_kernel, whose launches read the 7.6 GB of stored logits per step)
# the segment sums of the embedding backward only: ROLE 0 instantiations (ROLE 1 = the classifier one-hot dW)
K12 = ('spmm_kernel', 'spmm_pf_kernel', 'spmm_nc_kernel', 'combine_kernel', 'embed_fwd_kernel', 'embed_fwd_rows_kernel', 'seg_chunk_kernel<64, 0>',
       'seg_split1_kernel<64, 0>', 'seg_split2_kernel<64, 0>')
PMC_STEPS = 3


def per_kernel(path, counter, names=K5):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        name = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name'])
        for k in names:
            # (names of the bf16-table instantiations stay mangled: a plain substring test there)
            if (k in name) if ('<' in k or name.startswith('_Z')) else re.search(r'\b' + k + r'\b', name):
                vals[k].append(float(r['Counter_Value']) * 1e3)  # KB -> B
    return vals


if prec == 'c5':
    K5 = ()
fe = per_kernel(f'{pre}_fetch/run_counter_collection.csv', 'FETCH_SIZE')
wr = per_kernel(f'{pre}_write/run_counter_collection.csv', 'WRITE_SIZE')
rows = {}
# per HEAD: a head's dW sweep can take two launches (whole rounds + the split remainder, losshead.dw_plan), so every
# kernel's bytes are divided by the number of heads profiled (= the fwd_u sweep launches), not by its own launches
heads = max(1, len(fe[K5[0]])) if K5 else 1
for k in K5:
    f = 2 * sum(fe[k]) / heads
    w = sum(wr[k]) / heads
    rows[k] = dict(launches=len(fe[k]), fetch_bytes=round(f), write_bytes=round(w), bytes=round(f + w))
    print(f'{k:16} launches {len(fe[k]):3d}  per head: fetch {f / 1e6:9.1f} MB  write {w / 1e6:8.1f} MB')
tot = sum(r['bytes'] for r in rows.values())
print(f'K5 per head (fwd_u + rows + dw launches, {heads} heads): {tot / 1e6:.1f} MB')
# MFMA-busy fraction of the K5 kernels from the SQ pass (SQ_VALU_MFMA_BUSY_CYCLES over the 1024 SIMDs'
# cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs), summed over their launches
mfma_busy = None
try:
    busy, cyc = 0.0, 0.0
    for r in csv.DictReader(open(f'{pre}_sq/run_counter_collection.csv')):
        name = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name'])
        if not any((k in name) if '<' in k else re.search(r'\b' + k + r'\b', name) for k in K5):
            continue
        if r['Counter_Name'] == 'SQ_VALU_MFMA_BUSY_CYCLES':
            busy += float(r['Counter_Value'])
        elif r['Counter_Name'] == 'GRBM_GUI_ACTIVE':
            cyc += 1024 * float(r['Counter_Value']) / 8
    mfma_busy = round(busy / cyc, 4) if cyc else None
    print(f'K5 MFMA busy: {mfma_busy}')
except FileNotFoundError:
    pass
rev = subprocess.run(['git', 'rev-parse', '--short', 'HEAD'], capture_output=True, text=True).stdout.strip()
if out and prec != 'c5':
    rev = subprocess.run(['git', 'rev-parse', '--short', 'HEAD'], capture_output=True, text=True).stdout.strip()
    json.dump(dict(bytes_per_head=tot, bytes_per_launch_triple=tot, per_kernel=rows, mfma_busy=mfma_busy,
                   source=f'rocprofv3 --pmc FETCH_SIZE (x2) / WRITE_SIZE passes, {pre.split("/")[-1]}, rev {rev}'),
              open(out, 'w'), indent=1)

fe2 = per_kernel(f'{pre}_fetch/run_counter_collection.csv', 'FETCH_SIZE', K12)
wr2 = per_kernel(f'{pre}_write/run_counter_collection.csv', 'WRITE_SIZE', K12)
rows2 = {}
for k in K12:
    f = 2 * sum(fe2[k]) / PMC_STEPS
    w = sum(wr2[k]) / PMC_STEPS
    rows2[k] = dict(launches_per_step=len(fe2[k]) / PMC_STEPS, fetch_bytes=round(f), write_bytes=round(w),
                    bytes=round(f + w))
    print(f'{k:18} per step: fetch {f / 1e6:9.1f} MB  write {w / 1e6:8.1f} MB')
tot2 = sum(r['bytes'] for r in rows2.values())
print(f'K1+K2 per step: {tot2 / 1e6:.1f} MB')
if out:
    import os
    json.dump(dict(bytes_per_step=tot2, per_kernel=rows2,
                   source=f'rocprofv3 --pmc FETCH_SIZE (x2) / WRITE_SIZE passes, {pre.split("/")[-1]}, rev {rev}'),
              open(out if prec == 'c5' else
                   os.path.join(os.path.dirname(out), 'hbm_traffic.json' if prec == 'bf16' else 'hbm_traffic_fp32.json'),
                   'w'), indent=1)
