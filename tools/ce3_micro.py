"""Micro-benchmark of the fp32-mode K5 kernels (csrc/ce3.hip, split-bf16 ×3) at one head of the MB config
(n = 63,937 items, Mv ≈ 18.9k valid stacked rows, d = 256), HIP-event timed, next to the bf16 kernels of
ce.hip on the same shape.  Credited flops: 2·Mv·n·d per product (fwd_u: logits + U; dw: dW — the
recomputed logits and the two extra MFMAs of every split product are not credited).
usage: python tools/ce3_micro.py [Mv] [n] [split_fwd] [split_dw]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402
from c2dsr_amd.losshead import split_count  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
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
    Mp, n_pad = -(-Mv // 64) * 64, -(-n // 128) * 128 + 64
    n32 = -(-n // 32) * 32
    Hx = torch.empty(Mp, 2 * d, device=dev, dtype=torch.bfloat16)
    Wx = torch.empty(n32, 2 * d, device=dev, dtype=torch.bfloat16)
    t_split = timeit(lambda: (lib('c2dsr_f32_split_bf16', H, Mv, d, Mp, Hx, s),
                              lib('c2dsr_f32_split_bf16', W, n, d, n32, Wx, s)))
    bias2 = torch.empty(n_pad, **f32)
    lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
    tgt = torch.randint(0, n, (Mv,), device=dev)
    padc = torch.randn(Mv, **f32)
    lse, lse2, rows = torch.empty(Mv, **f32), torch.empty(Mp, **f32), torch.empty(Mv, **f32)
    ns = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) else split_count(Mv, 128)
    pm, ps = torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, **f32)
    Up = torch.empty(ns, Mv, d, **f32)
    fwd = lambda: lib('c2dsr_ce3_fused_fwd_u', Hx, Wx, bias2, Mv, n, d, ns, pm, ps, Up, padc, tgt, H, W, bias,  # noqa
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
            lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, full, d, 0, crow, gW, gb, s)
            lib('c2dsr_ce3_fused_dw', Hx, Wx.view(-1)[full * 2 * d:], bias2[full:], Mv, rem, d, k, crow, rWp, rbp, s)
            lib('c2dsr_sum_parts', rWp, k, rem * d, 1.0, gW.view(-1)[full * d:], s)
            lib('c2dsr_sum_parts', rbp, k, rem, 1.0, gb[full:], s)
    elif nr == -1:
        dw = lambda: lib('c2dsr_ce3_fused_dw_sk', Hx, Wx, bias2, Mv, n, d, crow, dWp[0], dbp[0], sk_ws, wsb, s)  # noqa: E731
    else:
        dw = lambda: lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, n, d, nr, crow, dWp, dbp, s)  # noqa: E731
    t_w = timeit(dw)
    t_s = timeit(lambda: lib('c2dsr_sum_parts', dWp, nr, n * d, 1.0, W, s)) if nr > 1 else 0.0  # (stream-K: the combine runs inside dw)
    fl = 2.0 * Mv * n * d
    print(f'ce3 Mv={Mv} n={n}: split {t_split:.1f} us; fwd_u {t_f:.1f} us ({2 * fl / t_f / 1e6:.0f} TFLOP/s credited, '
          f'{6 * fl / t_f / 1e6:.0f} executed, ns {ns}); dw {t_w:.1f} us ({fl / t_w / 1e6:.0f} credited, '
          f'{6 * fl / t_w / 1e6:.0f} executed, nr {nr}, sum {t_s:.1f} us); checksum {float(lse.sum()):.4f} {float(dWp.sum()):.4f}',
          flush=True)
    print_stamps([('fwd_u', fwd), ('dw', dw)])


def print_stamps(fns):
    """Diagnostic build (-DCE3_STAMP): cycles per tile per wave of the ce3 tile loop's phases."""
    import ctypes
    from c2dsr_amd import _lib
    so = ctypes.CDLL(os.path.join(_lib._DIR, 'libc2dsr_hip.so'))  # the stamp entry exists in the diagnostic build only
    if not hasattr(so, 'c2dsr_ce3_stamps'):
        return
    fn = so.c2dsr_ce3_stamps
    buf = (ctypes.c_ulonglong * 8)()
    ph = ('rescale/pre', 'S+epi', 'nop+dmawait', 'barrier', 'U+prep', 'loop-top')
    for name, f in fns:
        torch.cuda.synchronize()
        fn(buf, 1)
        f()
        torch.cuda.synchronize()
        fn(buf, 1)
        tiles = max(1, buf[6])
        print(f'  stamps {name}: ' + ', '.join(f'{p} {buf[i] / tiles:.0f}' for i, p in enumerate(ph))
              + f' (cycles per tile per wave, {tiles} wave-tiles)', flush=True)

if __name__ == '__main__':
    main()
