"""Effective clock and cycles per dispatch from a rocprofv3 --pmc GRBM_GUI_ACTIVE counter CSV (the
MI355X guide's DVFS recipe: clock ≈ GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time).
usage: python tools/clk_pmc.py <counter_collection.csv> [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ''
agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for r in rows:
    if sub not in r['Kernel_Name']:
        continue
    key = (r['Kernel_Name'][:70], int(r['Dispatch_Id']))
    agg[key][r['Counter_Name']] += float(r['Counter_Value'])
    meta[key] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
for key in sorted(agg, key=lambda k: k[1]):
    v, ns = agg[key], meta[key]
    cyc = v.get('GRBM_GUI_ACTIVE', 0) / 8
    extra = ' '.join(f'{k}={x:.4g}' for k, x in v.items() if k != 'GRBM_GUI_ACTIVE')
    print(f'{key[1]:5d} {key[0][:60]:60s} {ns / 1e3:9.1f} us  Mcyc {cyc / 1e6:7.3f}  GHz {cyc / ns:5.3f}  {extra}')
