"""Instruction mix of a kernel's hottest basic-block run in a hipcc --save-temps .s file (CPU only, no GPU).

    python tools/isa_stats.py FILE.s SUBSTRING [--dump]

Finds the function whose symbol contains SUBSTRING, splits it into basic blocks, and reports for the block
range with the most MFMAs (the tile loop) the counts of MFMAs, s_nop cycles, accvgpr moves, LDS reads, VALU
and waitcnts, plus the distribution of non-MFMA instructions between consecutive MFMAs.  --dump prints the
loop's instruction stream with MFMAs marked."""
import re
import sys
from collections import Counter


def function_body(text, sub):
    for m in re.finditer(r'^(\S+):\s*;\s*@\1\s*$', text, re.M):
        if sub in m.group(1):
            end = text.index('.Lfunc_end', m.end())
            return m.group(1), text[m.end():end]
    raise SystemExit(f'no function matching {sub}')


def blocks(body):
    out, cur, name = [], [], 'entry'
    for raw in body.split('\n'):
        line = raw.split(';')[0].strip()
        if not line:
            continue
        if line.endswith(':'):
            out.append((name, cur))
            name, cur = line[:-1], []
        elif not line.startswith('.'):
            cur.append(line)
    out.append((name, cur))
    return out


def main():
    path, sub = sys.argv[1], sys.argv[2]
    name, body = function_body(open(path).read(), sub)
    bl = blocks(body)
    # the loop: the largest-MFMA block that a later branch jumps back to
    best = max(bl, key=lambda b: sum(1 for i in b[1] if i.startswith('v_mfma')))
    # include the blocks from the loop head to the back-branch
    names = [b[0] for b in bl]
    head = best[0]
    for i, (n, ins) in enumerate(bl):
        for x in ins:
            m = re.match(r's_cbranch_\w+\s+(\S+)|s_branch\s+(\S+)', x)
            tgt = m and (m.group(1) or m.group(2))
            if tgt and tgt in names and names.index(tgt) <= names.index(head) and i >= names.index(head):
                head = tgt
                last = i
    i0 = names.index(head)
    i1 = max(names.index(best[0]), locals().get('last', names.index(best[0])))
    ins = [x for b in bl[i0:i1 + 1] for x in b[1]]
    op = lambda x: x.split()[0]
    c = Counter(op(x) for x in ins)
    nop = sum(int(x.split()[1]) + 1 for x in ins if op(x) == 's_nop')
    mf = [k for k, x in enumerate(ins) if op(x).startswith('v_mfma')]
    gaps = Counter(b - a - 1 for a, b in zip(mf, mf[1:]))
    print(f'{name[:90]}\nloop blocks {names[i0]}..{names[i1]}: {len(ins)} instructions, {len(mf)} MFMA, '
          f's_nop cycles {nop}, accvgpr {sum(v for k, v in c.items() if "accvgpr" in k)}, '
          f'ds_read {sum(v for k, v in c.items() if k.startswith("ds_read"))}, '
          f'VALU {sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith(("v_mfma", "v_accvgpr")))}, '
          f'waitcnt {c["s_waitcnt"]}, barrier {c["s_barrier"]}')
    print('instructions between consecutive MFMAs:', dict(sorted(gaps.items())))
    print('top ops:', c.most_common(18))
    if '--dump' in sys.argv:
        for x in ins:
            print(('>> ' if op(x).startswith('v_mfma') else '   ') + x)


if __name__ == '__main__':
    main()
