"""Fused loss head of ``Trainer.train_batch`` (trainer.py:85-156) as one autograd node.

forward:  masked-mean pooling (cal_mask, :85-108) → bilinear discriminators D_a/D_b
          (:104-108) → 4× BCE-with-logits (:113-119) → last-R slices and the four
          classifier heads with the pad column (:122-140) → 4× cross-entropy with
          ignore_index = pad column (:143-152) → count-weighted share loss, loss_rec,
          loss = λ·rec + (1-λ)·mi (:147-156).
backward: all gradients of the five encoder outputs; parameter gradients are
          accumulated directly into the parameters' ``.grad`` buffers.

The two heads that share a classifier matrix (share_a + specific_a, share_b +
specific_b) are stacked into one [2·B·R, d] GEMM each.  The logits are
materialised ([2BR, n+1] fp32, the pad column written by a row-dot); the
backward turns them into dlogits in place.
"""
from __future__ import annotations

import os

import torch
from torch.autograd import Function

from ._lib import error_word, lib, stage_ops, stream
from .ops import BF16, FP32, IndexPlan, _grad_target, index_plans, colsum, gemm, rg_kind, rgemm, weight_img, wg_kind, wgemm

FUSED_HEAD = True  # the training step's loss head on the c2dsr:: stage operators (csrc_torch/losshead_ops.cpp)
# fp32 mode, opt-in (C2DSR_CE_LOGITS=1): the forward sweep stores the logits (Mv·n fp32 per head: 4.9 GB at the
# Movie-Book head b) and the dW sweep reads them instead of recomputing them (c2dsr_ce3_fused_dw_lg*: one split product
# per tile instead of two); heads whose logits would exceed CE_LOGITS_GB keep the recomputing sweep.  Measured in the
# step (round 6): the dW sweeps −1.0 ms, the forward's 7.6 GB of stores +0.9 ms — not the default
CE_LOGITS = os.environ.get('C2DSR_CE_LOGITS', '1') != '0'
CE_LOGITS_GB = float(os.environ.get('C2DSR_CE_LOGITS_GB', '48'))


def keep_logits(Mv, n, mode):
    return int(bool(CE_LOGITS and mode == 0 and Mv > 0 and
                    -(-Mv // 128) * 128 * -(-n // 32) * 32 * 4 <= CE_LOGITS_GB * 2 ** 30))


_NCU = None


def _ncu():
    global _NCU
    if _NCU is None:
        _NCU = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count \
            if torch.cuda.is_available() else 256
    return _NCU


_GEOM = {}


def ce3_geometry(x3):
    """(stationary rows per workgroup, swept rows per LDS tile) of the fused-CE sweep kernels (csrc/ce3.hip
    c2dsr_ce3_geometry, a build-time choice): fp32 mode (split-bf16, x3) 128 / 32; bf16 mode 128 / 64 (CE3B_SBW /
    CE3B_T3: 3 stationary blocks × 32-row tiles = 192 / 32 measured slower in round 6)."""
    if x3 not in _GEOM:
        g = lib.raw('c2dsr_ce3_geometry')
        _GEOM[x3] = (int(g(int(bool(x3)), 0)), int(g(int(bool(x3)), 1)))
    return _GEOM[x3]


def split_count(rows, tile, max_split=16, per_cu=1):
    """Work splits for a (row tiles × splits) grid of one-workgroup-per-CU kernels: the count that
    minimises the launch's makespan ⌈tiles·s / slots⌉ / s (whole rounds of workgroups; a partial
    last round leaves CUs idle), the smaller count on ties (fewer partial slices to combine)."""
    tiles = max(1, -(-rows // tile))
    slots = _ncu() * per_cu
    best, best_t = 1, None
    for s in range(1, max_split + 1):
        t = -(-tiles * s // slots) / s
        if best_t is None or t < best_t - 1e-12:
            best, best_t = s, t
    return best


FWD_PLAN = True  # the forward split count from fwd_split_count's fitted cost (else split_count's whole-round fill)
# the bf16 kernels' fitted sweep costs (tools/ce3b_micro.py on the box; units: swept-tile times unless noted)
BF16_FIT = dict(fwd_wg=5.0, fwd_slab=2.7, dw_tile_us=1.47, dw_wg=9.0, dw_sk_loc=1.35)


def fwd_split_count(Mv, n, x3, d=256, max_split=16):
    """Column splits of the forward sweep (ce3.hip MODE 0: 128 stationary H rows per workgroup, the n columns in
    32-row tiles on split images, 64-row tiles on bf16 ones, split s ways) at d = 256: the least fitted cost
    rounds × (tiles per workgroup + a workgroup's fixed cost) + the U slabs' combine (c2dsr_ce_dh_from_u reads s slabs
    of Mv·d fp32), the smaller count on ties.  Fitted to fwd sweeps on the box (tools/ce3_micro.py / ce3b_micro.py,
    s = 3 … 16; fixed cost ≈ 4 / 5 tiles, a slab ≈ 2.1 / 2.7 tile-times at Mv = 18,944): fp32 Movie-Book head a
    (n = 36,845) 5 splits — 1614 µs against 1626 at 12, with 7 fewer 19 MB slabs —, head b (63,937) 12; bf16 5 for
    both (758 / 1239 µs against 793 / 1257 at 12), Food-Kitchen (Mv ≈ 9.5k) 3 (382 µs against 386 at 10, with 7
    fewer slabs).  Other widths: split_count (whole rounds)."""
    rb, rows = ce3_geometry(x3)
    if not (FWD_PLAN and d == 256):
        return split_count(Mv, rb, max_split)
    wg, slab = (4.0, 2.1) if x3 else (BF16_FIT['fwd_wg'], BF16_FIT['fwd_slab'])
    blocks = max(1, -(-Mv // rb))
    tiles = max(1, -(-n // rows))
    slots = _ncu()
    best, best_c = 1, None
    for s in range(1, max_split + 1):
        c = -(-blocks * s // slots) * (-(-tiles // s) + wg) + slab * s * Mv / 18944
        if best_c is None or c < best_c - 1e-9:
            best, best_c = s, c
    return best


def _dw_costs(n, Mv, x3, d=256, max_split=16):
    """Fitted cost (in swept-tile times) of the dW sweep (ce3.hip MODE 1: 128 stationary W rows per workgroup; the Mv
    swept rows in 32-row tiles on split images, 64-row tiles on bf16 ones) for each row-split count s — rounds ×
    (tiles per workgroup + a workgroup's fixed cost) + the partial slabs' combine — and for the stream-K sweep —
    (units per workgroup + fixed cost per segment) × a locality factor (its workgroups start at different swept
    tiles, so they share fewer of them in L2) + its combine.  Fitted to split / stream-K sweeps on the box
    (tools/ce3_micro.py / ce3b_micro.py: a tile 1.87 / 1.47 µs, a workgroup's fixed cost ≈ 16 / 9 tiles, a partial
    slab of n·d fp32 written and summed ≈ 7.5 µs at 36.8k × 256, stream-K locality 1.15 / 1.35)."""
    rb, rows = ce3_geometry(x3)
    tiles = max(1, -(-n // rb))
    sweep = max(1, -(-Mv // rows))
    t_tile, wg, sk_loc = (1.87, 16.0, 1.15) if x3 else (BF16_FIT['dw_tile_us'], BF16_FIT['dw_wg'], BF16_FIT['dw_sk_loc'])
    slab = 7.5 * (n * d) / (36845 * 256) / t_tile
    slots = _ncu()
    split = {}
    for s in range(1, max_split + 1):
        split[s] = -(-tiles * s // slots) * (-(-sweep // s) + wg) + (s * slab if s > 1 else 0.0)
    per = tiles * sweep / slots
    sk = sk_loc * (per + wg * (1.0 + per / sweep)) + 10.0 / t_tile
    return split, sk


def dw_split_count(n, Mv, x3, d=256, max_split=16):
    """Row splits of the dW sweep: the count of least fitted cost (_dw_costs), the smaller count on ties.  One split
    accumulates straight into the gradient.  (split_count alone picked 15 splits for the Food-Kitchen heads: 543 µs
    of sweep + sum where 3-4 take 379.)"""
    split, _ = _dw_costs(n, Mv, x3, d, max_split)
    best = min(split.values())
    return min(s for s in split if split[s] <= best + 1e-9)


DW_SK = True  # the dW sweep as stream-K (c2dsr_ce3*_fused_dw_sk) where its fitted cost is lower


def dw_plan(n, Mv, x3, d, both_grads=True):
    """The dW sweep's plan as the loss head's split argument (ce_head_backward's n_rsplit), the least fitted cost of
      k ≥ 1  row splits (dw_split_count; k = 1: one split added onto the gradients),
      0      stream-K (one workgroup per CU over equal ranges of (W row block, swept tile) units),
      −k     whole rounds of unsplit row blocks, then the last partial round's row blocks in k splits: the first
             ⌊blocks / CUs⌋·CUs row blocks added onto the gradients by one launch, the rest split k ways by a second —
             Movie-Book head a (288 row blocks on 256 CUs) and the Food-Kitchen heads (273) have a 32- / 17-block
             remainder that one undivided round would leave 7/8 of the chip idle for.
    Stream-K and the remainder split need both gradients and ce3.hip's kernels (d = 256: the fitted shapes; other
    widths keep split_count)."""
    rb, rows = ce3_geometry(x3)
    if d != 256:
        return split_count(n, rb)
    split, sk = _dw_costs(n, Mv, x3, d)
    best_k = dw_split_count(n, Mv, x3, d)
    plan, cost = best_k, split[best_k]
    if not (DW_SK and both_grads):
        return plan
    if sk < cost:
        plan, cost = 0, sk
    slots = _ncu()
    blocks = -(-n // rb)
    full = blocks // slots * slots
    if full and full < blocks:
        rem = n - full * rb
        rsplit, _ = _dw_costs(rem, Mv, x3, d)
        k = dw_split_count(rem, Mv, x3, d)
        sweep = max(1, -(-Mv // rows))
        t_wg = 16.0 if x3 else BF16_FIT['dw_wg']
        hyb = full // slots * (sweep + t_wg) + rsplit[k]
        if k > 1 and hyb < cost:
            plan, cost = -k, hyb
    return plan


def dw_full_rows(n, x3):
    """The W rows of the whole rounds of a remainder dW plan (dw_plan < 0): ⌊row blocks / CUs⌋·CUs row blocks, with
    the CU count the plan was costed on (ce_head_backward takes it as dw_full instead of re-deriving it)."""
    rb = ce3_geometry(x3)[0]
    return -(-n // rb) // _ncu() * _ncu() * rb


def ce_kind(precision, d):
    """Fused classifier-head kernels for this precision and width: 'b16' (ce.hip, bf16 operands), 'x3'
    (ce3.hip, split-bf16 operands: the fp32 mode), or None (materialised fp32 logits + exact fp32 GEMMs)."""
    if precision == BF16 and bool(lib.raw('c2dsr_ce_supported')(d)):
        return 'b16'
    if precision == FP32 and bool(lib.raw('c2dsr_ce3_supported')(d)):
        return 'x3'
    return None


def ce_entry(x3, d, role):
    """The fused head's sweep kernels: split-bf16 images → ce3.hip (x3); bf16 images → ce3.hip's plain-bf16
    instantiation where it covers d (128, 256), else ce.hip's pair (same arguments and outputs)."""
    if x3:
        return 'c2dsr_ce3_fused_' + role
    return ('c2dsr_ce3b_fused_' if bool(lib.raw('c2dsr_ce3_supported')(d)) else 'c2dsr_ce_fused_') + role


class LossMeta:
    def __init__(self, *, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, n_a, n_b, R, lam, Wa, ba, Wb, bb, wpad,
                 bpad, Da_w, Da_b, Db_w, Db_b, precision=FP32, B_global=None, allreduce=None, ce_pre=None,
                 row_sets=None, counts=None, reduce_async=None):
        """counts: (cnt [8] fp32, handle) — valid-target counts all-reduced ahead of the forward (data
        parallel); reduce_async(t) starts an all-reduce of t and returns its handle."""
        self.__dict__.update(locals())
        del self.__dict__['self']
        self.pending = None
        self.on_head_grads = None  # data parallel: called when the backward has written the head gradients
        self.after_first_ce = None  # host work to enqueue once the first long CE kernel is queued (or at the end)
        self.plan_state = None  # the step's plan cache when its target plans were built ahead (trainer.PLANS_EARLY)

    def run_after_first_ce(self):
        f, self.after_first_ce = self.after_first_ce, None
        if f is not None:
            f()

    def finish_values(self):
        """Data parallel: wait for the loss values' sums and recompute (loss, loss_rec, loss_mi) from them
        (the backward already ran on the gradient weights, which depend on the counts only)."""
        if self.pending is None:
            return
        work, vec, cnt, BR_global, out3 = self.pending
        self.pending = None
        work.wait()
        scratch = torch.empty(4, device=vec.device, dtype=torch.float32)
        lib('c2dsr_loss_finalize', vec, cnt, BR_global, float(self.lam), out3, scratch[:2], scratch[2:], stream())


def fused_head_mode(m, B, d, training):
    """0 / 1 (split-bf16 / bf16 operands) when the loss head runs on the stage operators: a training step with its
    targets compacted ahead (Trainer.prepare), the ce3.hip sweep kernels at this width and the projection kernels
    for the discriminators; None: op by op."""
    kind = ce_kind(m.precision, d)
    if not (FUSED_HEAD and training and m.ce_pre is not None and kind is not None
            and bool(lib.raw('c2dsr_ce3_supported')(d))):
        return None
    want = 'x3' if kind == 'x3' else 'b16'
    if rg_kind(m.precision, 2 * B, d, d) != want or wg_kind(m.precision, 2 * B, d, d) != want:
        return None
    return 0 if kind == 'x3' else 1


class LossHeadFn(Function):
    @staticmethod
    def forward(ctx, h_share, hx, hy, h_neg_a, h_neg_b, m: LossMeta):
        B, L = m.gm_a.shape  # (encoder outputs may hold a row subset: [n, d])
        d = h_share.shape[-1]
        mode = fused_head_mode(m, B, d, any(ctx.needs_input_grad[:5]))
        if mode is not None:
            return LossHeadFn._forward_stage(ctx, (h_share, hx, hy, h_neg_a, h_neg_b), m, mode)
        ctx.stage = None
        R = m.R
        BR = B * R
        dev = h_share.device
        s = stream()
        f32 = dict(device=dev, dtype=torch.float32)
        # ---- pooling (6 vectors) ----
        wa = torch.empty(B, L, **f32)
        wb = torch.empty(B, L, **f32)
        lib('c2dsr_pool_weights', m.gm_a, B, L, wa, s)
        lib('c2dsr_pool_weights', m.gm_b, B, L, wb, s)
        Phx = torch.empty(B, d, **f32)
        Phy = torch.empty(B, d, **f32)
        X2a = torch.empty(2 * B, d, **f32)  # [h_share·wb ; h_neg_a·wa]
        X2b = torch.empty(2 * B, d, **f32)  # [h_share·wa ; h_neg_b·wb]
        # encoder outputs may hold only the rows the loss reads (row_sets: share, a, b, neg_a, neg_b; the
        # last encoder layer ran on them): read through their inverse maps
        rsets = tuple(m.row_sets) if m.row_sets is not None else (None,) * 5
        mp = [r.inv if r is not None else None for r in rsets]
        lib('c2dsr_pool2_fwd', hx, mp[1], wa, None, B, L, d, Phx, None, s)
        lib('c2dsr_pool2_fwd', hy, mp[2], wb, None, B, L, d, Phy, None, s)
        lib('c2dsr_pool2_fwd', h_share, mp[0], wb, wa, B, L, d, X2a, X2b, s)  # both poolings of h_share (Q5)
        lib('c2dsr_pool2_fwd', h_neg_a, mp[3], wa, None, B, L, d, X2a[B:], None, s)
        lib('c2dsr_pool2_fwd', h_neg_b, mp[4], wb, None, B, L, d, X2b[B:], None, s)
        # ---- bilinear: s = x1ᵀ W x2 (+b)  via  U = X2·Wᵀ, s = rowdot(x1, U) ----
        Ua = torch.empty(2 * B, d, **f32)
        Ub = torch.empty(2 * B, d, **f32)
        for X2, Wd, U in ((X2a, m.Da_w, Ua), (X2b, m.Db_w, Ub)):
            kind = rg_kind(m.precision, 2 * B, d, d)
            if kind:  # the row-streaming MFMA GEMM (bf16 or split-bf16 operands)
                rgemm(X2, weight_img(Wd.view(d, d), kind), U, M=2 * B, N=d, K=d, x3=kind == 'x3',
                      frag=True)
            else:
                gemm(X2, Wd, U, M=2 * B, N=d, K=d, transB=1, precision=FP32)
        S = torch.empty(4, B, **f32)
        lib('c2dsr_mi_scores', Phx, Ua, m.Da_b, Phy, Ub, m.Db_b, B, d, S, s)  # the four scores, one launch
        vec = torch.empty(9, **f32)  # [CE sums ×4, counts ×4, loss_mi]
        Bg = m.B_global if m.B_global is not None else B
        dS = torch.empty(4, B, **f32)
        lib('c2dsr_mi_loss', S, B, Bg, vec[8:], dS, s)
        # ---- classifier heads ----
        kind = ce_kind(m.precision, d)
        fused = kind is not None
        x3 = kind == 'x3'  # fp32 mode: split-bf16 operands [rows][2d] = hi ‖ lo, three MFMAs per product
        ctx.fused, ctx.x3 = fused, x3
        heads = []
        specs = ((hx, m.Wa, m.ba, m.gt_share_a, m.gt_a, m.n_a), (hy, m.Wb, m.bb, m.gt_share_b, m.gt_b, m.n_b))
        M2 = 2 * BR
        pre = []
        pre_given = fused and m.ce_pre is not None  # targets + compaction enqueued by Trainer.prepare
        for k, (hdom, W, bias, t_share, t_spec, n) in enumerate(specs):
            Hcat = torch.empty(M2, d, **f32)
            Hpad = torch.empty(M2, d, **f32)
            lib('c2dsr_rec_gather', h_share, mp[0], hdom, mp[1 + k], B, L, d, R, Hcat, Hpad, s)
            comp = None
            if pre_given:
                tcat, idx, inv, tc, (hc, slot) = m.ce_pre[k]
                comp = (idx, inv, tc, (hc, slot))
                pre.append((Hcat, Hpad, tcat, comp))
                continue
            tcat = torch.empty(M2, device=dev, dtype=torch.int64)
            lib('c2dsr_rec_targets', t_share, t_spec, B, L, R, tcat, s)
            if fused:
                # rows whose target is the ignore index contribute nothing to the loss or any gradient
                # (trainer.py:131-154): the fused CE runs on the valid rows only (stable compaction)
                idx = torch.empty(M2, device=dev, dtype=torch.int32)
                inv = torch.empty(M2, device=dev, dtype=torch.int32)
                tc = torch.empty(M2, device=dev, dtype=torch.int64)
                cnt = torch.empty(2, device=dev, dtype=torch.int32)
                cws = torch.empty(lib.raw('c2dsr_compact_workspace')(M2, 1) // 4 + 1, device=dev,
                                  dtype=torch.int32)
                lib('c2dsr_compact_valid', tcat, M2, BR, n, idx, inv, tc, cnt, cws, error_word(), s)
                comp = (idx, inv, tc, cnt)
            pre.append((Hcat, Hpad, tcat, comp))
        if pre_given:  # deferred host read (ops.HostCounts), long since landed
            counts = [c[3][3][0][c[3][3][1] + j] for c in pre for j in (0, 1)]
        elif fused:  # one host read of both heads' valid-row counts (sizes the compact launches)
            counts = torch.cat([c[3][3] for c in pre]).tolist()
        for k, ((hdom, W, bias, t_share, t_spec, n), (Hcat, Hpad, tcat, comp)) in enumerate(zip(specs, pre)):
            lse = torch.empty(M2, **f32)
            rows = torch.empty(M2, **f32)
            if fused:
                idx, inv, tc, _ = comp
                Mv0, Mv1 = counts[2 * k], counts[2 * k + 1]
                Mv = Mv0 + Mv1
                M_pad = max(64, -(-Mv // 64) * 64)
                n_pad = -(-n // 128) * 128 + 64  # + a 64-value tail: tiles near n DMA 64 constants
                Hc = torch.empty(Mv, d, **f32)
                lib('c2dsr_gather_rows', Hcat, d, idx, Mv, d, Hc, s)
                if x3:  # hi ‖ lo images, zero rows past the end (whole 32-row tiles)
                    Hb = torch.empty(M_pad, 2 * d, device=dev, dtype=torch.bfloat16)
                    lib('c2dsr_f32_split_bf16', Hc, Mv, d, M_pad, Hb, s)
                    n32 = -(-n // 32) * 32
                    Wb = torch.empty(n32, 2 * d, device=dev, dtype=torch.bfloat16)
                    lib('c2dsr_f32_split_bf16', W, n, d, n32, Wb, s)
                else:
                    Hb = torch.empty(M_pad, d, device=dev, dtype=torch.bfloat16)  # whole 64-row H tiles (dW sweep)
                    if M_pad > Mv:
                        Hb[Mv:].zero_()
                    n64 = -(-n // 64) * 64  # whole 64-row W tiles for the LDS-DMA (zero rows past n)
                    Wb = torch.empty(n64, d, device=dev, dtype=torch.bfloat16)
                    if n64 > n:
                        Wb[n:].zero_()
                    if Mv:
                        lib('c2dsr_f32_to_bf16', Hc, Hc.numel(), Hb, s)
                    lib('c2dsr_f32_to_bf16', W, W.numel(), Wb, s)
                bias2 = torch.empty(n_pad, **f32)
                lib('c2dsr_ce_bias2', bias, n, n_pad, bias2, s)
                padlogit = torch.empty(M2, **f32)
                lib('c2dsr_rowdot', Hpad, d, m.wpad, 0, M2, d, m.bpad, padlogit, 1, s)
                padc = torch.empty(max(Mv, 1), **f32)
                lib('c2dsr_gather_rows', padlogit, 1, idx, Mv, 1, padc, s)
                lse_c = torch.empty(max(Mv, 1), **f32)
                rows_c = torch.empty(max(Mv, 1), **f32)
                lse2 = torch.empty(M_pad, **f32)
                u = None
                if Mv and (x3 or any(ctx.needs_input_grad[:5])):
                    # forward + the softmax part of the input gradient in one sweep (online lse, flash
                    # style): the backward runs no dH sweep
                    ns = fwd_split_count(Mv, n, x3, d) if ce_entry(x3, d, 'fwd_u').startswith('c2dsr_ce3') \
                        else split_count(Mv, 128)
                    pm = torch.empty(ns, Mv, **f32)
                    ps = torch.empty(ns, Mv, **f32)
                    Up = torch.empty(ns, Mv, d, **f32)
                    fa = (Hb, Wb, bias2, Mv, n, d, ns, pm, ps, Up, padc, tc, Hc, W, bias, lse_c, lse2, rows_c)
                    lg = None
                    if x3 and W.requires_grad and keep_logits(Mv, n, 0):  # the dW sweep reads the stored logits
                        lg = torch.empty(int(lib.raw('c2dsr_ce3_logits_floats')(Mv, n)), **f32)
                        lib('c2dsr_ce3_fused_fwd_u_lg', *fa, lg, s)
                    else:
                        lib(ce_entry(x3, d, 'fwd_u'), *fa, s)
                    u = (Up, pm, ns, lg)
                    m.run_after_first_ce()
                elif Mv:
                    ns = split_count(Mv, 256)
                    pm = torch.empty(ns, Mv, **f32)
                    ps = torch.empty(ns, Mv, **f32)
                    lib('c2dsr_ce_fused_fwd', Hb, Wb, bias2, Mv, n, d, ns, pm, ps, padc, tc, Hc, W, bias, lse_c,
                        lse2, rows_c, s)
                lib('c2dsr_expand_rows', rows_c, inv, M2, 1, rows, s)  # per-row losses, 0 on ignored rows
                # target sort for the one-hot part of dW/db, on the side stream under the rest of the step
                tplan = IndexPlan(tc[:Mv], n + 1) if Mv and any(ctx.needs_input_grad[:5]) and W.requires_grad else None
                heads.append((Hcat, Hpad, tcat, (Hb, Wb, padc, lse2, bias2, tplan, Hc, tc, inv, Mv, Mv0, lse_c, u), lse,
                              rows, W, bias, n))
            else:
                ld = n + 1
                logits = torch.empty(M2, ld, **f32)
                gemm(Hcat, W, logits, M=M2, N=n, K=d, transB=1, ldc=ld, bias=bias, precision=m.precision)
                lib('c2dsr_rowdot', Hpad, d, m.wpad, 0, M2, d, m.bpad, logits[:, n:], ld, s)
                lib('c2dsr_ce_fwd', logits, ld, M2, ld, tcat, n, lse, rows, s)
                heads.append((Hcat, Hpad, tcat, logits, lse, rows, W, bias, n))
        out3 = torch.empty(3, **f32)
        coefA = torch.empty(2, **f32)
        coefB = torch.empty(2, **f32)
        (_, _, tA, _, _, rA, _, _, _), (_, _, tB, _, _, rB, _, _, _) = heads
        lpw = torch.empty(max(1, int(lib.raw('c2dsr_loss_partials_workspace')(BR))), **f32)
        lib('c2dsr_loss_partials', rA, tA, m.n_a, rB, tB, m.n_b, BR, vec, lpw, s)
        cnt = None
        if m.counts is not None:
            # data parallel: the global valid-target counts (the only global values the gradient needs)
            # were all-reduced ahead of the forward (Trainer.prepare); the loss values' sums are reduced
            # asynchronously and finalized after the backward (LossMeta.finish_values)
            cnt, work = m.counts
            work.wait()
            # the collective works on its own copy: the loss finalised below (and returned) reads vec now
            vred = vec.clone()
            m.pending = (m.reduce_async(vred), vred, cnt, Bg * R, out3)
        elif m.allreduce is not None:  # data parallel without pre-reduced counts: reduce everything now
            m.allreduce(vec)
        lib('c2dsr_loss_finalize', vec, cnt, Bg * R, float(m.lam), out3, coefA, coefB, s)
        ctx.m, ctx.heads, ctx.coefs = m, heads, (coefA, coefB)
        ctx.mi = (Phx, Phy, X2a, X2b, Ua, Ub, dS)
        ctx.w = (wa, wb)
        ctx.shape = (B, L, d)
        ctx.rsets = rsets
        ctx.hshapes = [t.shape for t in (h_share, hx, hy, h_neg_a, h_neg_b)]
        loss, loss_rec, loss_mi_o = out3[0], out3[1], out3[2]
        ctx.mark_non_differentiable(loss_rec, loss_mi_o)
        ctx.set_materialize_grads(False)  # no zero scalars for the two reported losses
        m.run_after_first_ce()
        return loss, loss_rec, loss_mi_o

    @staticmethod
    def _forward_stage(ctx, hs, m, mode):
        """The forward on the stage operators: loss_disc_forward, ce_head_forward per head (the host work queued after
        the first head's long sweep: m.after_first_ce), loss_partials, loss_finalize (and the data-parallel
        reductions between them, as in the op-by-op path)."""
        T = stage_ops()
        B, L = m.gm_a.shape
        d = hs[0].shape[-1]
        R = m.R
        BR = B * R
        kind = 'x3' if mode == 0 else 'b16'
        rsets = tuple(m.row_sets) if m.row_sets is not None else (None,) * 5
        mp = [r.inv if r is not None else None for r in rsets]
        Bg = m.B_global if m.B_global is not None else B
        vec = torch.empty(9, device=hs[0].device, dtype=torch.float32)  # [CE sums ×4, counts ×4, loss_mi]
        D = [m.Da_w, m.Da_b, m.Db_w, m.Db_b]
        Dimg = [weight_img(m.Da_w.view(d, d), kind), weight_img(m.Db_w.view(d, d), kind)]
        disc = T.loss_disc_forward(list(hs), mp, m.gm_a, m.gm_b, D, Dimg, mode, Bg, vec)
        heads = []
        specs = ((hs[1], m.Wa, m.ba, m.n_a), (hs[2], m.Wb, m.bb, m.n_b))
        for k, (hdom, W, bias, n) in enumerate(specs):
            tcat, idx, inv, tc, (hc, slot) = m.ce_pre[k]
            Mv0, Mv1 = int(hc[slot]), int(hc[slot + 1])
            Mv = Mv0 + Mv1
            out = T.ce_head_forward(hs[0], mp[0], hdom, mp[1 + k], B, L, R, W, bias, m.wpad, m.bpad, idx, inv, tc,
                                    Mv0, Mv1, fwd_split_count(Mv, n, mode == 0, d), mode,
                                    keep_logits(Mv, n, mode) if W.requires_grad else 0)
            if k == 0:
                m.run_after_first_ce()
            # target sort for the one-hot part of dW/db, on the side stream under the rest of the step (or built with
            # the step's other plans ahead of the forward: trainer.PLANS_EARLY)
            tplan = None
            if Mv and W.requires_grad:
                tplan = index_plans(m.plan_state, [(tc[:Mv], n + 1)])[0] if m.plan_state is not None \
                    else IndexPlan(tc[:Mv], n + 1)
            heads.append((out[0], tcat, out[1:], inv, tc, Mv0, Mv1, tplan, W, bias, n))
        T.loss_partials(heads[0][0], heads[0][1], m.n_a, heads[1][0], heads[1][1], m.n_b, BR, vec)
        cnt = None
        if m.counts is not None:  # data parallel: global counts reduced ahead; the values' sums reduced async
            cnt, work = m.counts
            work.wait()
            vred = vec.clone()
            m.pending = (m.reduce_async(vred), vred, cnt, Bg * R, torch.empty(3, device=vec.device))
        elif m.allreduce is not None:
            m.allreduce(vec)
        out3, coefA, coefB = T.loss_finalize(vec, cnt, Bg * R, float(m.lam))
        if m.pending is not None:  # finish_values rewrites the returned losses in place
            m.pending = m.pending[:4] + (out3,)
        ctx.stage = (mode, kind, disc, [h[2:] for h in heads], (coefA, coefB), rsets, mp, (B, L, d))
        ctx.m = m
        loss, loss_rec, loss_mi_o = out3[0], out3[1], out3[2]
        ctx.mark_non_differentiable(loss_rec, loss_mi_o)
        ctx.set_materialize_grads(False)
        m.run_after_first_ce()
        return loss, loss_rec, loss_mi_o

    @staticmethod
    def _backward_stage(ctx, gloss):
        """ce_head_backward per head, then loss_disc_backward (discriminators, poolings, the heads' dH scatter)."""
        T = stage_ops()
        m = ctx.m
        mode, kind, disc, heads, coefs, rsets, mp, (B, L, d) = ctx.stage
        gscale = gloss.contiguous().reshape(1)
        gwpad, gbpad = _grad_target(m.wpad), _grad_target(m.bpad)
        hd = []
        for (saved, inv, tc, Mv0, Mv1, tplan, W, bias, n), coef in zip(heads, coefs):
            gW, gb = _grad_target(W), _grad_target(bias)
            nr = dw_plan(n, Mv0 + Mv1, mode == 0, d, gW is not None and gb is not None)
            hd += T.ce_head_backward(saved, W, inv, tc, Mv0, Mv1, coef, gscale, float(m.lam), gW, gb, gwpad, gbpad,
                                     tplan.get() if tplan is not None else None, nr, mode,
                                     dw_full_rows(n, mode == 0) if nr < 0 else 0)
        imgT = [weight_img(m.Da_w.view(d, d), kind, trans=True), weight_img(m.Db_w.view(d, d), kind, trans=True)]
        gD = [_grad_target(t) for t in (m.Da_w, m.Da_b, m.Db_w, m.Db_b)]
        sub = [r.idx[:r.n] if r is not None else None for r in rsets]
        dh = T.loss_disc_backward(disc, gscale, float(m.lam), [m.Da_w, m.Da_b, m.Db_w, m.Db_b], imgT, gD, hd, m.wpad,
                                  sub, mp, L, m.R, mode)
        if m.on_head_grads is not None:  # the classifier / discriminator gradients are final: their
            m.on_head_grads()                # collectives run under the encoder backwards (dp.py)
            m.on_head_grads = None
        ctx.m = ctx.stage = None
        return tuple(dh) + (None,)

    @staticmethod
    def backward(ctx, gloss, _g1, _g2):
        if ctx.stage is not None:
            return LossHeadFn._backward_stage(ctx, gloss)
        m = ctx.m
        B, L, d = ctx.shape
        R = m.R
        BR = B * R
        dev = gloss.device
        s = stream()
        f32 = dict(device=dev, dtype=torch.float32)
        gscale = gloss.contiguous().reshape(1)
        # ---- classifier heads ----
        # (first: their CE kernels are the long ones, so the host's bookkeeping for the discriminators and the
        # pooling below runs while they execute; the heads' input gradients are added after the pooling writes)
        scat = []
        rsets = ctx.rsets
        mp = [r.inv if r is not None else None for r in rsets]
        gwpad, gbpad = _grad_target(m.wpad), _grad_target(m.bpad)
        for k, ((Hcat, Hpad, tcat, logits, lse, rows, W, bias, n), coef) in enumerate(zip(ctx.heads, ctx.coefs)):
            M2 = 2 * BR
            dHcat = torch.empty(M2, d, **f32)
            gW, gb = _grad_target(W), _grad_target(bias)
            if ctx.fused:
                Hb, Wb, padc, lse2, bias2, tplan, Hc, tc, inv, Mv, Mv0, lse_c, u = logits
                M_pad = lse2.shape[0]
                rw = torch.empty(M_pad, **f32)
                t32 = torch.empty(M_pad, device=dev, dtype=torch.int32)
                dpad_c = torch.empty(max(Mv, 1), **f32)
                crow = torch.empty(M_pad + 64, **f32)  # + the tail the dW sweep's row-constant DMA reads
                dHc = torch.empty(max(Mv, 1), d, **f32)
                if Mv:
                    # compact rows keep their order: the first Mv0 are the shared-sequence rows (coef[0])
                    lib('c2dsr_ce_row_weights', tc, Mv, M_pad, n, coef, Mv0, gscale, float(m.lam), padc, lse_c, rw,
                        t32, lse2, crow, dpad_c, s)
                    lg = None
                    if u is not None:  # dH = rw·(softmax·W − W[t]) from the forward's online partials
                        Up, pm, nsu, lg = u
                        lib('c2dsr_ce_dh_from_u', Up, pm, nsu, Mv, d, lse2, t32, rw, W, n, dHc, s)
                    else:
                        ns = split_count(Mv, 128)
                        dHp = torch.empty(ns, Mv, d, **f32)
                        lib('c2dsr_ce_fused_dh', Hb, Wb, bias2, Mv, n, d, ns, crow, dHp, s)
                        lib('c2dsr_ce_dh_combine', dHp, ns, Mv, d, t32, rw, W, n, dHc, s)
                        del dHp
                    entry = ce_entry(ctx.x3, d, 'dw')
                    both = gW is not None and gb is not None and entry.startswith('c2dsr_ce3')
                    nr = dw_plan(n, Mv, ctx.x3, d, both)
                    ic = (2 if ctx.x3 else 1) * d

                    def dw(nsplit, o1, o2, off=0, rows=n):  # the sweep over W rows [off, off + rows)
                        if lg is not None:
                            lib('c2dsr_ce3_fused_dw_lg', Hb, lg, Mv, n, off, rows, d, nsplit, crow, o1, o2, s)
                        else:
                            lib(entry, Hb, Wb.view(-1)[off * ic:], bias2[off:], Mv, rows, d, nsplit, crow, o1, o2, s)
                    if nr == 0:  # stream-K: whole row blocks added onto the gradients, split ones combined in order
                        wsb = int(lib.raw('c2dsr_ce3_dw_sk_workspace')(d))
                        ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
                        if lg is not None:
                            lib('c2dsr_ce3_fused_dw_lg_sk', Hb, lg, Mv, n, d, crow, gW, gb, ws, wsb, s)
                        else:
                            lib(entry + '_sk', Hb, Wb, bias2, Mv, n, d, crow, gW, gb, ws, wsb, s)
                        del ws
                    elif nr < 0:  # whole rounds unsplit onto the gradients, the remainder row blocks −nr ways
                        full = dw_full_rows(n, ctx.x3)
                        rem, k = n - full, -nr
                        dw(0, gW, gb, 0, full)
                        dWp = torch.empty(k, rem, d, **f32)
                        dbp = torch.empty(k, rem, **f32)
                        dw(k, dWp, dbp, full, rem)
                        lib('c2dsr_sum_parts', dWp, k, rem * d, 1.0, gW.view(-1)[full * d:], s)
                        lib('c2dsr_sum_parts', dbp, k, rem, 1.0, gb[full:], s)
                        del dWp, dbp
                    elif nr == 1 and both:
                        # one split: the sweep adds onto the gradients itself (n_rsplit = 0; no partials / sum)
                        dw(0, gW, gb)
                    else:
                        dWp = torch.empty(nr, n, d, **f32)
                        dbp = torch.empty(nr, n, **f32)
                        dw(nr, dWp, dbp)
                        if gW is not None:
                            lib('c2dsr_sum_parts', dWp, nr, n * d, 1.0, gW, s)
                        if gb is not None:
                            lib('c2dsr_sum_parts', dbp, nr, n, 1.0, gb, s)
                        del dWp, dbp
                    if (gW is not None or gb is not None) and tplan is not None:
                        wsb = int(lib.raw('c2dsr_ce_onehot_planned_workspace')(Mv, n, d))
                        ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
                        lib('c2dsr_ce_onehot_dw_planned', tplan.get(), Mv, n, Hc, d, rw, gW, gb, ws, wsb, s)
                    elif gW is not None or gb is not None:
                        wsb = int(lib.raw('c2dsr_ce_onehot_workspace')(Mv, n, d))
                        ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
                        lib('c2dsr_ce_onehot_dw', tc, Mv, n, Hc, d, rw, gW, gb, ws, wsb, s)
                lib('c2dsr_expand_rows', dHc, inv, M2, d, dHcat, s)  # 0 on ignored rows
                dpad = torch.empty(M2, **f32)
                lib('c2dsr_expand_rows', dpad_c, inv, M2, 1, dpad, s)
                pad_col, pad_ld = dpad, 1
            else:
                ld = n + 1
                lib('c2dsr_ce_bwd', logits, ld, M2, ld, tcat, n, lse, coef, BR, gscale, float(m.lam), s)
                gemm(logits, W, dHcat, M=M2, N=d, K=n, lda=ld, precision=m.precision)
                if gW is not None:
                    gemm(logits, Hcat, gW, M=n, N=d, K=M2, transA=1, lda=ld, beta=1.0, precision=m.precision)
                if gb is not None:
                    colsum(logits, M2, n, ld, gb)
                pad_col, pad_ld = logits[:, n:], ld
            if gwpad is not None:  # gwpad[0, :] += Σ_r pad_col[r]·Hpad[r, :]
                ws = torch.empty(lib.raw('c2dsr_colsum_workspace')(M2, d), dtype=torch.uint8, device=dev)
                lib('c2dsr_wcolsum', Hpad, M2, d, d, pad_col, pad_ld, 1.0, 1.0, gwpad, ws, s)
            if gbpad is not None:
                colsum(pad_col, M2, 1, pad_ld, gbpad)
            scat.append((dHcat, pad_col, pad_ld, k))
        # ---- discriminators ----
        Phx, Phy, X2a, X2b, Ua, Ub, dS = ctx.mi
        lib('c2dsr_scale_ds', dS, 4 * B, gscale, float(1.0 - m.lam), s)
        dP = {}
        dx1s = [torch.empty(B, d, **f32) for _ in range(2)]
        dUs = [torch.empty(2 * B, d, **f32) for _ in range(2)]
        lib('c2dsr_bilinear_ds', Ua, Ub, Phx, Phy, dS, B, d, dx1s[0], dx1s[1], dUs[0], dUs[1], s)
        for (x1, X2, U, Wd, bd, k) in ((Phx, X2a, Ua, m.Da_w, m.Da_b, 0), (Phy, X2b, Ub, m.Db_w, m.Db_b, 2)):
            dx1, dU = dx1s[k // 2], dUs[k // 2]
            dX2 = torch.empty(2 * B, d, **f32)
            kind = rg_kind(m.precision, 2 * B, d, d)
            b16 = kind is not None and wg_kind(m.precision, 2 * B, d, d) is not None
            if b16:
                rgemm(dU, weight_img(Wd.view(d, d), kind, trans=True), dX2, M=2 * B, N=d, K=d, x3=kind == 'x3',
                      frag=True)
            else:
                gemm(dU, Wd, dX2, M=2 * B, N=d, K=d, precision=FP32)
            gWd = _grad_target(Wd)
            if gWd is not None and b16:  # not deferred: the head range is reduced as this backward returns
                wgemm(dU, X2, gWd.view(d, d), T=2 * B, N=d, D=d, defer=False, x3=kind == 'x3')
            elif gWd is not None:
                gemm(dU, X2, gWd, M=d, N=d, K=2 * B, transA=1, beta=1.0, precision=FP32)
            gbd = _grad_target(bd)
            if gbd is not None:
                colsum(dS[k], 2 * B, 1, 1, gbd)
            dP[k] = (dx1, dX2)
        (dPhx, dX2a), (dPhy, dX2b) = dP[0], dP[2]
        wa, wb = ctx.w
        # the pooling backward WRITES the five encoder-output gradients (no zero fill); the classifier
        # heads below add their last-R-position parts
        # (row-subset outputs get row-subset gradients: pooling writes their rows, heads add through the maps)
        dh_share, dhx, dhy, dh_na, dh_nb = [torch.empty(sh, **f32) for sh in ctx.hshapes]
        sub = [(r.idx, r.n) if r is not None else (None, 0) for r in rsets]
        lib('c2dsr_pool2_bwd', dPhx, wa, None, None, B, L, d, *sub[1], 0, dhx, s)
        lib('c2dsr_pool2_bwd', dPhy, wb, None, None, B, L, d, *sub[2], 0, dhy, s)
        lib('c2dsr_pool2_bwd', dX2a, wb, dX2b, wa, B, L, d, *sub[0], 0, dh_share, s)
        lib('c2dsr_pool2_bwd', dX2a[B:], wa, None, None, B, L, d, *sub[3], 0, dh_na, s)
        lib('c2dsr_pool2_bwd', dX2b[B:], wb, None, None, B, L, d, *sub[4], 0, dh_nb, s)
        for dHcat, pad_col, pad_ld, k in scat:
            # classifier_pad's input gradient (pad column ⊗ wpad) is folded into the scatter
            lib('c2dsr_rec_scatter', dHcat, pad_col, pad_ld, m.wpad, B, L, d, R, dh_share, mp[0], (dhx, dhy)[k],
                mp[1 + k], s)
        # the saved buffers (bf16 images, logits / lse, plans) are released with the backward even if a
        # caller keeps the graph alive (e.g. an undetached loss accumulator)
        if m.on_head_grads is not None:  # the classifier / discriminator gradients are final: their
            m.on_head_grads()                # collectives run under the encoder backwards (dp.py)
            m.on_head_grads = None
        ctx.m = ctx.heads = ctx.mi = ctx.w = ctx.rsets = ctx.coefs = None
        return dh_share, dhx, dhy, dh_na, dh_nb, None
