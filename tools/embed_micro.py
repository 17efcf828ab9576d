"""Micro-benchmark of the K2 embedding backward pieces at bench sizes (GPU box):
G-only (item segment sums), gP-only (position sums), both, and the index plan build.
Synthetic batch shaped like bench.py's MB workload (Zipf items, ~45 % padding rows)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402
from c2dsr_amd.ops import IndexPlan  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    B, L, d = 2048, 50, 256
    N = 100783
    rng = np.random.default_rng(1)
    lens = rng.integers(6, L + 1, size=B)
    seq = np.full((B, L), N - 1, dtype=np.int64)
    pos = np.zeros((B, L), dtype=np.int64)
    for b in range(B):
        n = lens[b]
        seq[b, L - n:] = np.minimum(rng.zipf(1.2, size=n) - 1, N - 2)
        pos[b, L - n:] = np.arange(1, n + 1) % L
    n_rows = B * L
    dev = torch.device('cuda')
    sd, pd = torch.from_numpy(seq).to(dev), torch.from_numpy(pos).to(dev)
    gX = torch.randn(n_rows, d, device=dev)
    G = torch.zeros(N, d, device=dev)
    gP = torch.zeros(L, d, device=dev)
    sp, pp = IndexPlan(sd, N), IndexPlan(pd, L)
    spb, ppb = sp.get(), pp.get()
    wsb = lib.raw('c2dsr_embed_bwd_planned_workspace')(n_rows, d)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    uniq = int(torch.unique(sd).numel())
    s = stream()

    def run(g, p):
        lib('c2dsr_embed_bwd_planned', spb if g is not None else None, ppb if p is not None else None, n_rows, d, gX,
            0, 0, 0.0, 0, 1.0, g, N, p, L, None, ws, wsb, s)

    t_g = timeit(lambda: run(G, None))
    t_p = timeit(lambda: run(None, gP))
    t_b = timeit(lambda: run(G, gP))
    pb = int(lib.raw('c2dsr_index_plan_bytes')(n_rows))
    buf = torch.empty(pb, dtype=torch.uint8, device=dev)
    t_plan = timeit(lambda: lib('c2dsr_index_plan', sd, n_rows, N, buf, pb, None, s))
    byt = n_rows * (16 + 4 * d) + 8 * d * uniq
    print(f'rows {n_rows} uniq {uniq}: G-only {t_g:.1f} us, gP-only {t_p:.1f} us, both {t_b:.1f} us '
          f'({byt / (t_b * 1e-6) / 1e9:.0f} GB/s credited), seq plan build {t_plan:.1f} us', flush=True)

    # the fused pass's form (c2dsr_embed_bwd_planned_rows): the gradient as two compact parts — the rows the loss reads
    # (here: every non-padding row with probability 0.6) and the padding rows (the keys of the inverted mask)
    nonpad = pos.reshape(-1) != 0
    q_rows = np.flatnonzero(nonpad & (rng.random(n_rows) < 0.6))
    k_rows = np.flatnonzero(~nonpad)
    inv_a = np.full(n_rows, -1, dtype=np.int32)
    inv_b = np.full(n_rows, -1, dtype=np.int32)
    inv_a[q_rows] = np.arange(q_rows.size, dtype=np.int32)
    inv_b[k_rows] = np.arange(k_rows.size, dtype=np.int32)
    gXa = torch.randn(q_rows.size, d, device=dev)
    gXb = torch.randn(k_rows.size, d, device=dev)
    ia, ib = torch.from_numpy(inv_a).to(dev), torch.from_numpy(inv_b).to(dev)

    def run_rows(g, p):
        lib('c2dsr_embed_bwd_planned_rows', spb if g is not None else None, ppb if p is not None else None, n_rows, d,
            gXa, ia, gXb, ib, 0, 0, 0.0, 0, 1.0, g, N, p, L, ws, wsb, s)

    r_g = timeit(lambda: run_rows(G, None))
    r_p = timeit(lambda: run_rows(None, gP))
    r_b = timeit(lambda: run_rows(G, gP))
    print(f'two-part rows (q {q_rows.size}, k {k_rows.size}): G-only {r_g:.1f} us, gP-only {r_p:.1f} us, both {r_b:.1f} us '
          f'({byt / (r_b * 1e-6) / 1e9:.0f} GB/s credited); checksum {float(G.sum()):.4e} {float(gP.sum()):.4e}',
          flush=True)


if __name__ == '__main__':
    main()
