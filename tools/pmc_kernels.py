"""Per-kernel sums of every counter in a rocprofv3 --pmc CSV (run_counter_collection.csv), averaged per launch.

    python tools/pmc_kernels.py DIR [SUBSTRING ...]

DIR is the -d directory of the rocprofv3 run (-o run --output-format csv); only kernels whose name contains one of
the substrings are printed (all when none given).  Ratios printed for the LDS counters when present:
bank-conflict cycles / LDS-array cycles, and the MFMA-busy share of the wave cycles."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    subs = sys.argv[2:]
    files = glob.glob(f'{d}/**/run_counter_collection.csv', recursive=True) + glob.glob(f'{d}/run_counter_collection.csv')
    if not files:
        raise SystemExit(f'no run_counter_collection.csv under {d}')
    val = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name'])
            name = re.sub(r'\(.*', '', name)
            if subs and not any(s in name for s in subs):
                continue
            val[name][r['Counter_Name']] += float(r['Counter_Value'])
            disp[name].add((f, r.get('Dispatch_Id', '')))
    for name, cs in sorted(val.items()):
        n = max(1, len(disp[name]))
        print(f'{name[:80]}  ({n} launches)')
        for c, v in sorted(cs.items()):
            print(f'    {c:28s} {v / n:16.1f}')
        if cs.get('SQ_LDS_IDX_ACTIVE'):
            print(f'    bank-conflict share of LDS-array cycles: {cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_LDS_IDX_ACTIVE"]:.3f}')
        if cs.get('SQ_BUSY_CYCLES') and cs.get('SQ_VALU_MFMA_BUSY_CYCLES'):
            print(f'    MFMA busy / SQ busy (x1/1024 SIMDs not applied): '
                  f'{cs["SQ_VALU_MFMA_BUSY_CYCLES"] / cs["SQ_BUSY_CYCLES"]:.3f}')


if __name__ == '__main__':
    main()
