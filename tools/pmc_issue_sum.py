"""Per-kernel sums of the tools/pmc_issue.sh passes (TAG_a, TAG_b), per launch, with the issue split
normalised to SQ_WAVE_CYCLES.  usage: python tools/pmc_issue_sum.py gpurun_out/TAG [kernel-substring]"""
import csv
import re
import sys
from collections import defaultdict

pre = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ''
tot = defaultdict(lambda: defaultdict(float))
nd = defaultdict(set)
for part in ('a', 'b'):
    for r in csv.DictReader(open(f'{pre}_{part}/run_counter_collection.csv')):
        k = re.sub(r'\(.*', '', re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name']))[:60]
        if pat not in k:
            continue
        tot[k][r['Counter_Name']] += float(r['Counter_Value'])
        nd[k].add((part, r['Dispatch_Id']))
for k, c in tot.items():
    n = max(1, len([d for d in nd[k] if d[0] == 'a']))
    wc = c.get('SQ_WAVE_CYCLES', 0) or 1
    print(k, f'launches {n}')
    for name in sorted(c):
        v = c[name]
        print(f'   {name:28s} {v / n:14.4g}  /wave_cyc {v / wc:.3f}')
