"""Per-kernel summary of the tools/pmc.sh passes: HBM bytes per launch (FETCH_SIZE doubled per the
gfx950 correction in MI355X_MICROARCH.md §HBM, WRITE_SIZE as is) and the SQ issue/stall split.
usage: python tools/pmc_summary.py gpurun_out/TAG   (reads TAG_fetch, TAG_write, TAG_sq)"""
import csv
import re
import sys
from collections import defaultdict

pre = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25


def short(n):
    n = re.sub(r'\(anonymous namespace\)::', '', n)
    return re.sub(r'\(.*', '', n)[:48]


def load(path):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    dur = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = short(r['Kernel_Name'])
        per[k][r['Counter_Name']].append(float(r['Counter_Value']))
        dur[k][r['Dispatch_Id']] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    return per, dur


fe, dur = load(f'{pre}_fetch/run_counter_collection.csv')
wr, _ = load(f'{pre}_write/run_counter_collection.csv')
sq, _ = load(f'{pre}_sq/run_counter_collection.csv')
avg = lambda v: sum(v) / len(v) if v else 0.0
rows = []
for k in fe:
    t = sum(dur[k].values())
    rows.append((t, k))
rows.sort(reverse=True)
print(f'{"kernel":48} {"n":>4} {"us/launch":>9} {"fetchMB":>8} {"writeMB":>8} {"GB/s":>7} '
      f'{"mfma%":>6} {"wait%":>6} {"stall%":>6} {"lds%":>5} {"valu/wv":>8}')
for t, k in rows[:top]:
    n = len(dur[k])
    us = t / n / 1e3
    f = 2 * avg(fe[k].get('FETCH_SIZE', [])) / 1e3  # KB → MB (FETCH_SIZE is in KB) x2 correction
    w = avg(wr[k].get('WRITE_SIZE', [])) / 1e3
    s = sq.get(k, {})
    wc = avg(s.get('SQ_WAVE_CYCLES', [])) or 1.0
    bc = avg(s.get('SQ_BUSY_CYCLES', [])) or 1.0
    mf = avg(s.get('SQ_VALU_MFMA_BUSY_CYCLES', []))
    # MFMA busy fraction over the 1024 SIMDs: cycles from GRBM_GUI_ACTIVE (summed over the 8 XCDs)
    # when collected, else the launch duration at 2.1 GHz
    cyc = avg(s.get('GRBM_GUI_ACTIVE', [])) / 8 or us * 2.1e3
    print(f'{k:48} {n:4d} {us:9.1f} {f:8.1f} {w:8.1f} {(f + w) * 1e3 / us:7.0f} '
          f'{100 * mf / (1024 * cyc):6.1f} {100 * avg(s.get("SQ_WAIT_ANY", [])) / wc:6.1f} '
          f'{100 * avg(s.get("SQ_WAIT_INST_ANY", [])) / wc:6.1f} {100 * avg(s.get("SQ_WAIT_INST_LDS", [])) / wc:5.1f} '
          f'{avg(s.get("SQ_INSTS_VALU", [])):8.0f}')
