"""Micro-benchmark of the bf16-mode K5 kernels (csrc/ce3.hip plain-bf16 instantiation: c2dsr_ce3b_fused_fwd_u / _dw)
at one classifier head, HIP-event timed.  Credited flops 2·Mv·n·d per product (fwd_u: logits + U; dw: dW).
usage: python tools/ce3b_micro.py [Mv] [n] [split_fwd] [split_dw]   (defaults: the FK config's head b, B = 1024: Mv 9472,
       n 34,886; splits: losshead.split_count)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402
from c2dsr_amd.losshead import split_count  # noqa: E402
from tools.ce3_micro import print_stamps, timeit  # noqa: E402


def main():
    Mv = int(sys.argv[1]) if len(sys.argv) > 1 else 9472
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 34886
    d = 256
    dev = torch.device('cuda')
    torch.manual_seed(0)
    f32 = dict(device=dev, dtype=torch.float32)
    s = stream()
    H = torch.randn(Mv, d, **f32) * 0.5
    W = torch.randn(n, d, **f32) * 0.05
    bias = torch.randn(n, **f32) * 0.1
    Mp, n_pad, n64 = -(-Mv // 64) * 64, -(-n // 128) * 128 + 64, -(-n // 64) * 64
    Hb = torch.zeros(Mp, d, device=dev, dtype=torch.bfloat16)
    Wb = torch.zeros(n64, d, device=dev, dtype=torch.bfloat16)
    lib('c2dsr_f32_to_bf16', H, H.numel(), Hb, s)
    lib('c2dsr_f32_to_bf16', W, W.numel(), Wb, s)
    bias2 = torch.empty(n_pad, **f32)
    lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
    tgt = torch.randint(0, n, (Mv,), device=dev)
    padc = torch.randn(Mv, **f32)
    lse, lse2, rows = torch.empty(Mv, **f32), torch.empty(Mp, **f32), torch.empty(Mv, **f32)
    ns = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) else split_count(Mv, 128)
    pm, ps = torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, **f32)
    Up = torch.empty(ns, Mv, d, **f32)
    fwd = lambda: lib('c2dsr_ce3b_fused_fwd_u', Hb, Wb, bias2, Mv, n, d, ns, pm, ps, Up, padc, tgt, H, W, bias,  # noqa
                      lse, lse2, rows, s)
    t_f = timeit(fwd)
    rw, dpad = torch.empty(Mp, **f32), torch.empty(Mp, **f32)
    crow = torch.empty(Mp + 64, **f32)
    t32 = torch.empty(Mp, device=dev, dtype=torch.int32)
    coef = torch.tensor([1.0 / Mv, 1.0 / Mv], **f32)
    gscale = torch.ones(1, **f32)
    lib('c2dsr_ce_row_weights', tgt, Mv, Mp, n, coef, Mv // 2, gscale, 0.7, padc, lse, rw, t32, lse2, crow, dpad, s)
    nr = int(sys.argv[4]) if len(sys.argv) > 4 and int(sys.argv[4]) else split_count(n, 128)
    if nr == -1:  # stream-K (c2dsr_ce3*_fused_dw_sk) onto gradient buffers
        wsb = int(lib.raw('c2dsr_ce3_dw_sk_workspace')(d))
        sk_ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
        dWp, dbp = torch.zeros(1, n, d, **f32), torch.zeros(1, n, **f32)
    else:
        dWp, dbp = torch.empty(max(nr, 1), n, d, **f32), torch.empty(max(nr, 1), n, **f32)
    if nr <= -2:  # whole rounds of row blocks unsplit, the remainder split -nr ways (losshead.dw_plan's third form)
        from c2dsr_amd.losshead import _ncu
        full = -(-n // 128) // _ncu() * _ncu() * 128
        rem, k = n - full, -nr
        gW, gb = torch.zeros(n, d, **f32), torch.zeros(n, **f32)
        rWp, rbp = torch.empty(k, rem, d, **f32), torch.empty(k, rem, **f32)

        def dw():
            lib('c2dsr_ce3b_fused_dw', Hb, Wb, bias2, Mv, full, d, 0, crow, gW, gb, s)
            lib('c2dsr_ce3b_fused_dw', Hb, Wb.view(-1)[full * d:], bias2[full:], Mv, rem, d, k, crow, rWp, rbp, s)
            lib('c2dsr_sum_parts', rWp, k, rem * d, 1.0, gW.view(-1)[full * d:], s)
            lib('c2dsr_sum_parts', rbp, k, rem, 1.0, gb[full:], s)
    elif nr == -1:
        dw = lambda: lib('c2dsr_ce3b_fused_dw_sk', Hb, Wb, bias2, Mv, n, d, crow, dWp[0], dbp[0], sk_ws, wsb, s)  # noqa: E731
    else:
        dw = lambda: lib('c2dsr_ce3b_fused_dw', Hb, Wb, bias2, Mv, n, d, nr, crow, dWp, dbp, s)  # noqa: E731
    t_w = timeit(dw)
    t_s = timeit(lambda: lib('c2dsr_sum_parts', dWp, nr, n * d, 1.0, W, s)) if nr > 1 else 0.0  # (stream-K: the combine runs inside dw)
    fl = 2.0 * Mv * n * d
    print(f'ce3b Mv={Mv} n={n}: fwd_u {t_f:.1f} us ({2 * fl / t_f / 1e6:.0f} TFLOP/s, ns {ns}); dw {t_w:.1f} us '
          f'({2 * fl / t_w / 1e6:.0f} executed, {fl / t_w / 1e6:.0f} credited, nr {nr}, sum {t_s:.1f} us); both {3 * fl / (t_f + t_w) / 1e6:.0f} '
          f'credited = {3 * fl / (t_f + t_w) / 1e6 / 2500:.3f} of 2.5 PF; checksum {float(lse.sum()):.4f} '
          f'{float(dWp.sum()):.4f}', flush=True)
    print_stamps([('fwd_u', fwd), ('dw', dw)])


if __name__ == '__main__':
    main()
