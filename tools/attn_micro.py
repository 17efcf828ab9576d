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
    pdrop = float(os.environ.get('ATTN_P', '0.2'))
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
    # row-subset layout (the last layer of a training pass): queries = last R positions + ~30% of the rest,
    # keys = the padding rows
    need = rng.random((B, L)) < 0.3
    need[:, -10:] = True

    def rowset(mask):
        flat = mask.reshape(-1)
        idx = np.nonzero(flat)[0].astype(np.int32)
        off = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
        return torch.from_numpy(idx).to(dev), torch.from_numpy(off).to(dev), len(idx)
    qi, qo, nq = rowset(need)
    ki, ko, nk = rowset(seq == pad)
    q = torch.randn(nq, d, device=dev)
    kv = torch.randn(nk, 2 * d, device=dev)
    o_r = torch.empty(nq, d, device=dev)
    do_r = torch.randn(nq, d, device=dev)
    dq = torch.empty(nq, d, device=dev, dtype=torch.bfloat16)
    dkv = torch.empty(nk, 2 * d, device=dev, dtype=torch.bfloat16)
    fr = lambda: lib('c2dsr_attn_fwd_rows', q, kv, sd, pad, qi, qo, ki, ko, B, L, d, H, 1, 2, pdrop, 0, o_r, P, s)  # noqa
    gr = lambda: lib('c2dsr_attn_bwd_rows', q, kv, sd, pad, qi, qo, ki, ko, B, L, d, H, 1, 2, pdrop, 0, P, do_r,  # noqa
                     dq, dkv, 1, s)
    tfr = timeit(fr)
    tbr = timeit(gr)
    # the fp32 mode's backward (fp32 dq / dkv: attn_bwd_rows<float>)
    dq32 = torch.empty(nq, d, device=dev)
    dkv32 = torch.empty(nk, 2 * d, device=dev)
    gr32 = lambda: lib('c2dsr_attn_bwd_rows', q, kv, sd, pad, qi, qo, ki, ko, B, L, d, H, 1, 2, pdrop, 0, P, do_r,  # noqa
                       dq32, dkv32, 0, s)
    tbr32 = timeit(gr32)
    print(f'{os.path.basename(os.environ.get("C2DSR_LIB", "default"))}: attn fwd {tf:.1f} us, bwd {tb:.1f} us; '
          f'rows (nq {nq / B:.1f}, nk {nk / B:.1f} per seq) fwd {tfr:.1f} us, bwd {tbr:.1f} us (bf16 out) '
          f'{tbr32:.1f} us (fp32 out); checksum {float(o_r.double().sum()):.6e} {float(dkv.double().sum()):.6e}',
          flush=True)
    # a domain pass's shape (the a / b sequences: most positions are the other domain's, i.e. padding keys)
    lens2 = rng.integers(2, 26, size=B)
    seq2 = np.full((B, L), pad, dtype=np.int64)
    for b in range(B):
        pos2 = np.sort(rng.choice(L, size=lens2[b], replace=False))
        seq2[b, pos2] = rng.integers(0, pad, size=lens2[b])
    sd2 = torch.from_numpy(seq2).to(dev)
    need2 = (rng.random((B, L)) < 0.2) | (seq2 != pad)
    need2[:, -10:] = True
    qi2, qo2, nq2 = rowset(need2 & (rng.random((B, L)) < 0.55))
    ki2, ko2, nk2 = rowset(seq2 == pad)
    q2 = torch.randn(nq2, d, device=dev)
    kv2 = torch.randn(nk2, 2 * d, device=dev)
    o2 = torch.empty(nq2, d, device=dev)
    do2 = torch.randn(nq2, d, device=dev)
    dq2 = torch.empty(nq2, d, device=dev)
    dkv2 = torch.empty(nk2, 2 * d, device=dev)
    f2 = lambda: lib('c2dsr_attn_fwd_rows', q2, kv2, sd2, pad, qi2, qo2, ki2, ko2, B, L, d, H, 1, 2, pdrop, 0, o2, P, s)  # noqa
    g2 = lambda: lib('c2dsr_attn_bwd_rows', q2, kv2, sd2, pad, qi2, qo2, ki2, ko2, B, L, d, H, 1, 2, pdrop, 0, P, do2,  # noqa
                     dq2, dkv2, 0, s)
    print(f'  domain-pass shape (nq {nq2 / B:.1f}, nk {nk2 / B:.1f} per seq): fwd {timeit(f2):.1f} us, '
          f'bwd {timeit(g2):.1f} us (fp32 out)', flush=True)


if __name__ == '__main__':
    main()
