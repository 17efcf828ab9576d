"""Micro-benchmark of K5's stored-logits path (csrc/ce3.hip: c2dsr_ce3_fused_fwd_u_lg + c2dsr_ce3_fused_dw_lg*) against
the recomputing sweeps (c2dsr_ce3_fused_fwd_u + c2dsr_ce3_fused_dw*) at the Movie-Book heads (fp32 mode, d = 256),
HIP-event timed, with the dW / db of both paths compared (max-abs difference over the gradient's max-abs).
usage: python tools/ce3_lg_micro.py [Mv] [n ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402
from c2dsr_amd.losshead import dw_full_rows, dw_plan, fwd_split_count  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def head(Mv, n, d=256):
    dev = torch.device('cuda')
    torch.manual_seed(0)
    f32 = dict(device=dev, dtype=torch.float32)
    s = stream()
    H = torch.randn(Mv, d, **f32) * 0.5
    W = torch.randn(n, d, **f32) * 0.05
    bias = torch.randn(n, **f32) * 0.1
    Mp, n_pad, n32 = -(-Mv // 64) * 64, -(-n // 128) * 128 + 64, -(-n // 32) * 32
    Hx = torch.empty(Mp, 2 * d, device=dev, dtype=torch.bfloat16)
    Wx = torch.empty(n32, 2 * d, device=dev, dtype=torch.bfloat16)
    lib('c2dsr_f32_split_bf16', H, Mv, d, Mp, Hx, s)
    lib('c2dsr_f32_split_bf16', W, n, d, n32, Wx, s)
    bias2 = torch.empty(n_pad, **f32)
    lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
    tgt = torch.randint(0, n, (Mv,), device=dev)
    padc = torch.randn(Mv, **f32)
    lse, lse2, rows = torch.empty(Mv, **f32), torch.empty(Mp, **f32), torch.empty(Mv, **f32)
    ns = fwd_split_count(Mv, n, True, d)
    pm, ps = torch.empty(ns, Mv, **f32), torch.empty(ns, Mv, **f32)
    Up = torch.empty(ns, Mv, d, **f32)
    lg = torch.empty(int(lib.raw('c2dsr_ce3_logits_floats')(Mv, n)), **f32)
    a = (Hx, Wx, bias2, Mv, n, d, ns, pm, ps, Up, padc, tgt, H, W, bias, lse, lse2, rows)
    t_f = timeit(lambda: lib('c2dsr_ce3_fused_fwd_u', *a, s))
    t_fl = timeit(lambda: lib('c2dsr_ce3_fused_fwd_u_lg', *a, lg, s))
    rw, dpad = torch.empty(Mp, **f32), torch.empty(Mp, **f32)
    crow = torch.empty(Mp + 64, **f32)
    t32 = torch.empty(Mp, device=dev, dtype=torch.int32)
    coef = torch.tensor([1.0 / Mv, 1.0 / Mv], **f32)
    gs = torch.ones(1, **f32)
    lib('c2dsr_ce_row_weights', tgt, Mv, Mp, n, coef, Mv, gs, 1.0, padc, lse, rw, t32, lse2, crow, dpad, s)
    wsb = int(lib.raw('c2dsr_ce3_dw_sk_workspace')(d))
    ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
    gW, gb = torch.zeros(n, d, **f32), torch.zeros(n, **f32)
    out = {}

    def run(kind, use_lg):
        if kind == 'sk':
            if use_lg:
                lib('c2dsr_ce3_fused_dw_lg_sk', Hx, lg, Mv, n, d, crow, gW, gb, ws, wsb, s)
            else:
                lib('c2dsr_ce3_fused_dw_sk', Hx, Wx, bias2, Mv, n, d, crow, gW, gb, ws, wsb, s)
            return
        k = int(kind)
        if k < 0:
            full = dw_full_rows(n, True)
            rem = n - full
            dWp, dbp = torch.empty(-k, rem, d, **f32), torch.empty(-k, rem, **f32)
            if use_lg:
                lib('c2dsr_ce3_fused_dw_lg', Hx, lg, Mv, n, 0, full, d, 0, crow, gW, gb, s)
                lib('c2dsr_ce3_fused_dw_lg', Hx, lg, Mv, n, full, rem, d, -k, crow, dWp, dbp, s)
            else:
                lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, full, d, 0, crow, gW, gb, s)
                lib('c2dsr_ce3_fused_dw', Hx, Wx.view(-1)[full * 2 * d:], bias2[full:], Mv, rem, d, -k, crow, dWp,
                    dbp, s)
            lib('c2dsr_sum_parts', dWp, -k, rem * d, 1.0, gW.view(-1)[full * d:], s)
            lib('c2dsr_sum_parts', dbp, -k, rem, 1.0, gb[full:], s)
        elif k <= 1:
            if use_lg:
                lib('c2dsr_ce3_fused_dw_lg', Hx, lg, Mv, n, 0, n, d, 0, crow, gW, gb, s)
            else:
                lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, n, d, 0, crow, gW, gb, s)
        else:
            dWp, dbp = torch.empty(k, n, d, **f32), torch.empty(k, n, **f32)
            if use_lg:
                lib('c2dsr_ce3_fused_dw_lg', Hx, lg, Mv, n, 0, n, d, k, crow, dWp, dbp, s)
            else:
                lib('c2dsr_ce3_fused_dw', Hx, Wx, bias2, Mv, n, d, k, crow, dWp, dbp, s)
            lib('c2dsr_sum_parts', dWp, k, n * d, 1.0, gW, s)
            lib('c2dsr_sum_parts', dbp, k, n, 1.0, gb, s)

    plan = dw_plan(n, Mv, True, d)
    kinds = ['1', '2', '3', 'sk'] + ([str(plan)] if plan < 0 else []) + (['-4', '-8'] if plan >= 0 else [])
    if os.environ.get('KINDS'):
        kinds = os.environ['KINDS'].split(',')
    for kind in kinds:
        for use_lg in (False, True):
            out[(kind, use_lg)] = timeit(lambda: run(kind, use_lg))
    # parity of the two dW paths (plan as the step runs it)
    res = []
    for use_lg in (False, True):
        gW.zero_()
        gb.zero_()
        run(str(plan) if plan != 0 else 'sk', use_lg)
        torch.cuda.synchronize()
        res.append((gW.clone(), gb.clone()))
    dw_rel = float((res[0][0] - res[1][0]).abs().max() / res[0][0].abs().max())
    db_rel = float((res[0][1] - res[1][1]).abs().max() / res[0][1].abs().max())
    fl = 2.0 * Mv * n * d
    print(f'head Mv={Mv} n={n}: fwd splits {ns}, dw plan {plan}, logits {lg.numel() * 4 / 1e9:.2f} GB')
    print(f'  fwd_u {t_f:8.1f} us   fwd_u_lg {t_fl:8.1f} us  (+{(t_fl / t_f - 1) * 100:.1f} %)  '
          f'{2 * fl / t_fl / 1e6:.1f} TF credited')
    for kind in kinds:
        a0, a1 = out[(kind, False)], out[(kind, True)]
        print(f'  dw[{kind:>3}] recompute {a0:8.1f} us   logits {a1:8.1f} us  ({a1 / a0:.3f}x)  '
              f'logits read {lg.numel() * 4 / a1 / 1e3:.0f} GB/s')
    print(f'  dW rel diff {dw_rel:.2e}  db rel diff {db_rel:.2e}', flush=True)
    return t_f, t_fl, out


def main():
    Mv = int(sys.argv[1]) if len(sys.argv) > 1 else 18944
    ns = [int(x) for x in sys.argv[2:]] or [63937, 36845]
    for n in ns:
        head(Mv, n)


if __name__ == '__main__':
    main()
