"""Micro-benchmark of the attention core at bench sizes (B=2048, L=50, d=256, H=1, dropout 0.2):
c2dsr_attn_fwd / c2dsr_attn_bwd, padding as in bench.py's synthetic sequences (left padding, n ~ U[6, L])."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402


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
    B, L, d, H = 2048, 50, 256, 1
    pad = 100782
    rng = np.random.default_rng(1)
    lens = rng.integers(6, L + 1, size=B)
    seq = np.full((B, L), pad, dtype=np.int64)
    for b in range(B):
        seq[b, L - lens[b]:] = rng.integers(0, pad, size=lens[b])
    dev = torch.device('cuda')
    sd = torch.from_numpy(seq).to(dev)
    qkv = torch.randn(B, L, 3 * d, device=dev)
    out = torch.empty(B, L, d, device=dev)
    P = torch.empty(int(lib.raw("c2dsr_attn_psave_floats")(B, L, d, H)), device=dev)  # the kernels' layout
    dout = torch.randn(B, L, d, device=dev)
    dqkv = torch.empty_like(qkv)
    s = stream()
    f = lambda: lib('c2dsr_attn_fwd', qkv, sd, pad, B, L, d, H, 1, 2, 0.2, 0, out, P, s)  # noqa: E731
    g = lambda: lib('c2dsr_attn_bwd', qkv, sd, pad, B, L, d, H, 1, 2, 0.2, 0, P, dout, dqkv, s)  # noqa: E731
    tf = timeit(f)
    tb = timeit(g)
    print(f'attn fwd {tf:.1f} us, bwd {tb:.1f} us ({os.environ.get("C2DSR_ATTN_TILED") and "tiled" or "default"})',
          flush=True)


if __name__ == '__main__':
    main()
