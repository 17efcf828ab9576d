"""Micro-benchmark of the K5 kernels at the bench's shapes: c2dsr_ce_fused_fwd_u (online lse + the softmax
part of dH) and c2dsr_ce_fused_dw, one head of the MB config (n = 63,937 items, Mv ≈ 18.9k valid stacked rows,
d = 256), HIP-event timed.  Compare kernel variants by pointing C2DSR_LIB at a variant library
(tools/ce_variants.sh builds them with the ce.hip tuning knobs).  Times both bf16 pairs: ce.hip's and ce3.hip's
plain-bf16 instantiation (c2dsr_ce3b_*).
usage: python tools/ce_micro.py [Mv] [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402
from c2dsr_amd.losshead import split_count  # noqa: E402


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
    Mv = int(sys.argv[1]) if len(sys.argv) > 1 else 18944
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 63937
    d = 256
    dev = torch.device('cuda')
    torch.manual_seed(0)
    f32 = dict(device=dev, dtype=torch.float32)
    s = stream()
    H = torch.randn(Mv, d, **f32) * 0.5
    W = torch.randn(n, d, **f32) * 0.05
    bias = torch.randn(n, **f32) * 0.1
    Mp, n_pad = -(-Mv // 64) * 64, -(-n // 64) * 64
    Hb = torch.zeros(Mp, d, device=dev, dtype=torch.bfloat16)
    Wb = torch.zeros(n_pad, d, device=dev, dtype=torch.bfloat16)
    lib('c2dsr_f32_to_bf16', H, Mv * d, Hb, s)
    lib('c2dsr_f32_to_bf16', W, n * d, Wb, s)
    bias2 = torch.empty(n_pad + 64, **f32)
    lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
    tgt = torch.randint(0, n, (Mv,), device=dev)
    padc = torch.randn(Mv, **f32)
    lse, lse2, rows = (torch.empty(Mv, **f32) for _ in range(3))
    ns = split_count(Mv, 128)
    pm, ps = torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, **f32)
    Up = torch.empty(ns, Mv, d, **f32)
    rw, crow, dpad = torch.empty(Mp, **f32), torch.empty(Mp + 64, **f32), torch.empty(Mp, **f32)
    t32 = torch.empty(Mp, device=dev, dtype=torch.int32)
    coef = torch.tensor([1.0 / Mv, 1.0 / Mv], **f32)
    gscale = torch.ones(1, **f32)
    nr = split_count(n, 128)
    dWp, dbp = torch.empty(nr, n, d, **f32), torch.empty(nr, n, **f32)
    fl = 2.0 * Mv * n * d
    for pre in ('c2dsr_ce_fused_', 'c2dsr_ce3b_fused_'):
        fwd = lambda: lib(pre + 'fwd_u', Hb, Wb, bias2, Mv, n, d, ns, pm, ps, Up, padc, tgt, H, W, bias,  # noqa
                          lse, lse2, rows, s)
        t_f = timeit(fwd)
        lib('c2dsr_ce_row_weights', tgt, Mv, Mp, n, coef, Mv // 2, gscale, 0.7, padc, lse, rw, t32, lse2, crow, dpad,
            s)
        dw = lambda: lib(pre + 'dw', Hb, Wb, bias2, Mv, n, d, nr, crow, dWp, dbp, s)  # noqa: E731
        t_w = timeit(dw)
        print(f'{os.path.basename(os.environ.get("C2DSR_LIB", "default"))} {pre[6:-7]}: fwd_u {t_f:.1f} us '
              f'({2 * fl / t_f / 1e6:.0f} TFLOP/s credited, ns {ns}), dw {t_w:.1f} us ({fl / t_w / 1e6:.0f} credited, '
              f'{2 * fl / t_w / 1e6:.0f} computed, nr {nr}); '
              f'checksum {float(lse.sum()):.4f} {float(dWp.sum()):.4f}', flush=True)
        if 'ce3b' in pre:
            from ce3_micro import print_stamps
            print_stamps([('fwd_u', fwd), ('dw', dw)])


if __name__ == '__main__':
    main()
