"""GPU idle time per training step from a rocprofv3 kernel trace.

usage: python tools/gaps.py gpurun_out/prof_TAG [n_gaps]

Steps are delimited by the AdamW kernel (one launch per step).  For each step: wall span, time with
at least one kernel running (union over all queues), and the largest idle gaps with the kernels
either side (host-bound stretches: syncs, Python launch overhead).
"""
import csv
import glob
import os
import sys


def load(d):
    path = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    return rows


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return name.split('(')[0][:48]


def main():
    d = sys.argv[1]
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows = load(d)
    ends = [e for s, e, n in rows if 'adamw_kernel' in n]
    for a, b in zip(ends[:-1], ends[1:]):
        ks = [(s, e, n) for s, e, n in rows if s >= a and e <= b]
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        prev = None
        for s, e, n in ks:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((s - cur_e, short(prev), short(n)))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = n
        if cur_e is not None:
            busy += cur_e - cur_s
        span = b - a
        print(f'step: span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms, '
              f'{len(ks)} kernels')
        for g, p, n in sorted(gaps, reverse=True)[:ng]:
            print(f'   {g / 1e3:8.1f} us  {p}  ->  {n}')


if __name__ == '__main__':
    main()
