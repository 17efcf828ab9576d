"""Can the K5 dW sweep (ce3_kernel MODE 1: one workgroup per CU, 135 KB LDS, 256 VGPRs per wave — half a SIMD's
register file) share the CUs with the step's memory-bound kernels that fit beside it (AdamW: 28 VGPRs, no LDS)?
Times, at the MB head-b shape (Mv = 18,944, n = 63,937, d = 256) and 80 M AdamW parameters (the step's parameters
outside the classifier heads), each alone and both enqueued at once on two streams (dW first).
usage: python tools/overlap_micro.py [adamw_params]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib  # noqa: E402


def timed(fn, reps=5):
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
    n_adam = int(sys.argv[1]) if len(sys.argv) > 1 else 80_000_000
    Mv, n, d = 18944, 63937, 256
    dev = torch.device('cuda')
    torch.manual_seed(0)
    f32 = dict(device=dev, dtype=torch.float32)
    s0 = torch.cuda.current_stream()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    H = torch.randn(Mv, d, **f32) * 0.5
    W = torch.randn(n, d, **f32) * 0.05
    bias = torch.randn(n, **f32) * 0.1
    Mp, n_pad, n32 = -(-Mv // 64) * 64, -(-n // 128) * 128 + 64, -(-n // 32) * 32
    Hx = torch.empty(Mp, 2 * d, device=dev, dtype=torch.bfloat16)
    Wx = torch.empty(n32, 2 * d, device=dev, dtype=torch.bfloat16)
    s = s0.cuda_stream
    lib('c2dsr_f32_split_bf16', H, Mv, d, Mp, Hx, s)
    lib('c2dsr_f32_split_bf16', W, n, d, n32, Wx, s)
    bias2 = torch.empty(n_pad, **f32)
    lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
    tgt = torch.randint(0, n, (Mv,), device=dev)
    padc = torch.randn(Mv, **f32)
    lse, lse2, rows = torch.empty(Mv, **f32), torch.empty(Mp, **f32), torch.empty(Mv, **f32)
    ns = 12
    pm, ps, Up = torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, d, **f32)
    lib('c2dsr_ce3_fused_fwd_u', Hx, Wx, bias2, Mv, n, d, ns, pm, ps, Up, padc, tgt, H, W, bias, lse, lse2, rows, s)
    rw, dpad = torch.empty(Mp, **f32), torch.empty(Mp, **f32)
    crow = torch.empty(Mp + 64, **f32)
    t32 = torch.empty(Mp, device=dev, dtype=torch.int32)
    coef = torch.tensor([1.0 / Mv, 1.0 / Mv], **f32)
    gscale = torch.ones(1, **f32)
    lib('c2dsr_ce_row_weights', tgt, Mv, Mp, n, coef, Mv // 2, gscale, 0.7, padc, lse, rw, t32, lse2, crow, dpad, s)
    gW, gb = torch.zeros(n, d, **f32), torch.zeros(n, **f32)
    buf = [torch.zeros(n_adam, **f32) for _ in range(5)]
    p, acc, m, v, vx = buf
    del Up, pm, ps
    torch.cuda.synchronize()

    def dw(st):
        lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, n, d, 0, crow, gW, gb, st.cuda_stream)

    def adam(st):
        lib('c2dsr_adamw', p, acc, acc, m, v, vx, n_adam, 1e-3, 5e-4, 0.9, 0.999, 1e-8, 1, None, st.cuda_stream)

    def both():
        ev = torch.cuda.Event()
        ev.record(s0)
        sa.wait_event(ev)
        sb.wait_event(ev)
        dw(sa)
        adam(sb)
        s0.wait_stream(sa)
        s0.wait_stream(sb)

    def both_late():  # AdamW enqueued after dW has started (the deferred sweep's order in a step)
        ev = torch.cuda.Event()
        ev.record(s0)
        sa.wait_event(ev)
        dw(sa)
        adam(s0)
        s0.wait_stream(sa)

    t_dw = timed(lambda: dw(s0))
    t_ad = timed(lambda: adam(s0))
    t_seq = timed(lambda: (dw(s0), adam(s0)))
    t_both = timed(both)
    t_late = timed(both_late)
    print(f'dW alone {t_dw:8.1f} us, AdamW ({n_adam / 1e6:.0f} M) alone {t_ad:7.1f} us, sequential {t_seq:8.1f} us, '
          f'two streams {t_both:8.1f} us, dW side + AdamW main {t_late:8.1f} us  (saved {t_seq - min(t_both, t_late):.1f})',
          flush=True)
    for k in (4, 8):  # the GCN-backward-like part: k row-streaming passes beside the sweep
        X = torch.randn(40_000_000 // k * k, **f32)
        Y = torch.empty_like(X)
        t_c = timed(lambda: [Y.copy_(X) for _ in range(k)])

        def cboth():
            ev = torch.cuda.Event()
            ev.record(s0)
            sa.wait_event(ev)
            dw(sa)
            for _ in range(k):
                Y.copy_(X)
            s0.wait_stream(sa)
        t_cb = timed(cboth)
        print(f'  + {k} copies of 160 MB: alone {t_c:8.1f} us, with dW on the side {t_cb:8.1f} us '
              f'(sequential {t_dw + t_c:8.1f})', flush=True)


if __name__ == '__main__':
    main()
