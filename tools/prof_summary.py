"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: per-kernel totals per step."""
import csv
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'{"ms/step":>9} {"calls":>6} {"avg_us":>9} {"%":>6}  kernel')
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:9.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} "
          f"{float(r['TotalDurationNs']) / tot * 100:6.1f}  {r['Name'][:100]}")
print(f'total kernel ms/step: {tot / 1e6 / steps:.2f}')
