"""Same-box A/B of a module-level switch on the default bench line: python tools/bench_ab.py MODULE.FLAG[,MODULE.FLAG] ROUNDS
(runs bench.py --no-cpu-baseline --no-extra in a child process per setting, alternating, ROUNDS times each)."""
import json
import os
import subprocess
import sys

flag, rounds = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
# FLAG may name several module attributes, comma-separated: they are switched together
sets = [f.rsplit('.', 1) for f in flag.split(',')]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = ("import sys, runpy; sys.argv = ['bench.py', '--no-cpu-baseline', '--no-extra']; "
        + "; ".join(f"import {m}; {m}.{a} = {{v}}" for m, a in sets)
        + "; runpy.run_path('bench.py', run_name='__main__')")
res = {True: [], False: []}
for r in range(rounds):
    for v in (True, False):
        out = subprocess.run([sys.executable, '-c', code.format(v=v)], cwd=root, capture_output=True,
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
