"""Same-box A/B of a module-level switch on the default bench line: python tools/bench_ab.py MODULE.FLAG ROUNDS
(runs bench.py --no-cpu-baseline --no-extra in a child process per setting, alternating, ROUNDS times each)."""
import json
import os
import subprocess
import sys

flag, rounds = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
mod, attr = flag.rsplit('.', 1)
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys, runpy; sys.argv = ['bench.py', '--no-cpu-baseline', '--no-extra']; import {m}; {m}.{a} = {v}; "
        "runpy.run_path('bench.py', run_name='__main__')")
res = {True: [], False: []}
for r in range(rounds):
    for v in (True, False):
        out = subprocess.run([sys.executable, '-c', code.format(m=mod, a=attr, v=v)], cwd=root, capture_output=True,
                             text=True, timeout=600)
        line = [x for x in out.stdout.splitlines() if x.startswith('{')]
        if out.returncode or not line:
            print(out.stdout[-2000:], out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(line[-1])
        res[v].append(d['value'])
        print(f'{flag}={v}: {d["value"]:.0f} seq/s, {d["ms_per_step"]:.3f} ms/step', flush=True)
for v in (True, False):
    print(f'{flag}={v}: mean {sum(res[v]) / len(res[v]):.0f} seq/s over {len(res[v])}')
