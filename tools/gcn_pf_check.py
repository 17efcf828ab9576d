"""Bit-identity probe for K1 variants on bf16 tables at d = 512 (the C5 width): forward (mask on the gathered
rows) and backward (Aᵀ, mask on the output rows) on a 400,001-row synthetic item graph with split hub rows;
prints a digest of both outputs and the per-launch time.  Run once per library (C2DSR_LIB_DIR=...) and compare."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd import graph as GR  # noqa: E402
from c2dsr_amd import ops, synth  # noqa: E402


def main():
    dev = torch.device('cuda')
    n_a = n_b = 200_000
    d, L = 512, 100
    N = n_a + n_b + 1
    items, off = synth.make_flat_sequences(40_000, n_a, n_b, L, seed=2)
    seq_id = np.repeat(np.arange(off.size - 1, dtype=np.int64), np.diff(off))
    same = seq_id[1:] == seq_id[:-1]
    g = GR.normalized_csr(np.stack([items[:-1][same], items[1:][same]], 1), N)
    dg = GR.DeviceGraph(g, dev)
    torch.manual_seed(0)
    E = torch.empty(N, d, device=dev, dtype=torch.bfloat16).normal_(0.0, 0.1)
    H, G = torch.empty_like(E), torch.empty_like(E)
    keys, p = (11, 22), 0.2
    f = lambda: ops.spmm(dg, False, E, keys, p, 0, 0.5, E, 0.5, 0.0, -1, 0.0, H)  # noqa: E731
    b = lambda: ops.spmm(dg, True, H, keys, p, 1, 0.5, H, 0.5, 1.0, N - 1, 1.0, G)  # noqa: E731
    G.zero_()
    f()
    b()
    torch.cuda.synchronize()
    dig = hashlib.sha1(H.view(torch.int16).cpu().numpy().tobytes() + G.view(torch.int16).cpu().numpy().tobytes())
    ts = []
    for fn in (f, b):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    print(f'{os.environ.get("C2DSR_LIB", "default")}: digest {dig.hexdigest()[:16]} fwd {ts[0]:.1f} us '
          f'bwd {ts[1]:.1f} us (n_work {dg.n_work}, n_split {dg.n_split})', flush=True)


if __name__ == '__main__':
    main()
