"""Host lead over the device per kernel, from one rocprofv3 run with --kernel-trace --hip-trace: for every kernel,
lead = kernel start − end of the host API call that launched it (joined on Correlation_Id).  A lead near zero means
the device waited for the host at that launch (the host is the bottleneck there); a large lead means the host was
that far ahead.  Per step (AdamW-delimited, as tools/gaps.py): the median / minimum lead, and the idle gaps whose
following kernel had a lead below 50 us (host-bound idle) versus the rest.
usage: python tools/host_lag.py gpurun_out/TAG_dir"""
import csv
import glob
import os
import statistics
import sys


def load(d, pat):
    path = glob.glob(os.path.join(d, '**', pat), recursive=True)
    return list(csv.DictReader(open(path[0]))) if path else []


def main():
    d = sys.argv[1]
    ks = load(d, '*kernel_trace.csv')
    api = {r['Correlation_Id']: r for r in load(d, '*hip_api_trace.csv')}
    rows = []
    for r in ks:
        a = api.get(r['Correlation_Id'])
        if a is None:
            continue
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(a['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    print(f'{len(rows)} kernels joined to their launch calls ({len(ks)} kernels, {len(api)} API records)')
    from collections import Counter
    cnt, tim = Counter(), Counter()
    for r in api.values():
        cnt[r['Function']] += 1
        tim[r['Function']] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    n_steps = max(1, sum(1 for r in rows if 'adamw_kernel' in r[3]))
    print(f'HIP API calls per step (of {n_steps} steps): count, host us')
    for f, c in cnt.most_common(15):
        print(f'   {f:40s} {c / n_steps:9.1f} {tim[f] / n_steps:9.1f}')
    ends = [i for i, x in enumerate(rows) if 'adamw_kernel' in x[3]]
    for a, b in zip(ends[:-1], ends[1:]):
        seg = rows[a + 1:b + 1]
        leads = [(s - h) / 1e3 for s, e, h, n in seg]
        host_idle, other_idle, prev_end = 0.0, 0.0, rows[a][1]
        for s, e, h, n in seg:
            if s > prev_end:
                gap = (s - prev_end) / 1e3
                if (s - h) / 1e3 < 50:
                    host_idle += gap
                else:
                    other_idle += gap
            prev_end = max(prev_end, e)
        print(f'step: lead median {statistics.median(leads):8.1f} us, min {min(leads):7.1f} us; idle after a '
              f'host-bound launch {host_idle:7.1f} us, other idle {other_idle:7.1f} us')


if __name__ == '__main__':
    main()
