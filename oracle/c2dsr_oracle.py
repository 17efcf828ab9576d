"""ORACLE — test infrastructure only.  CPU fp32 restatement of the C2DSR training
step of the reference (crystal22/C2DSR); never imported by the product path
(``c2dsr_amd``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it, and only as the checker / the CPU baseline.

Pinned against golden vectors produced by the reference itself
(``tools/gen_fixtures.py`` → ``tests/golden/model_*.npz``; see
``tests/test_oracle_golden.py``).  Written functionally over a flat parameter
dict keyed by the reference's ``state_dict`` names; gradients come from torch
autograd on CPU (plain fp32 reference, as for any floating-point kernel).

Reference semantics restated (file:line in /root/reference):
  * GCN                 models/encoders.py:36-48  (mean of [E, A·drop(E), ...], E undropped, Q12)
  * convolve_graph      models/C2DSR.py:59-62
  * embedding fuse      models/C2DSR.py:64-85     ((H[seq] + E[seq])·√d; F.embedding has no padding_idx, Q4)
  * SelfAttention       models/encoders.py:7-33   (+pos_emb, dropout, TransformerEncoder, final LN eps 1e-8)
      nn.TransformerEncoderLayer math path (n_head=1 ⇒ no fast path), causal mask +
      INVERTED key-padding mask (seq != pad masks real tokens, Q1); a fully masked row → 0 (Q2)
  * cal_mask / pooling  trainer.py:85-108         (cross-masked h_share pooling, Q5)
  * bilinear + BCE      trainer.py:104-119, C2DSR.py:46-55
  * heads + CE          trainer.py:121-154        (pad column = ignore_index, Q6; count weighting Q7; Q8)
  * loss / AdamW        trainer.py:156-158, :21-22 (amsgrad, decoupled wd; grads accumulate, Q3)
  * evaluate_batch      trainer.py:162-181        (rank vs sampled negatives, ties not counted)
  * cal_metrics/score   utils/metrics.py:4-31     (HR/MRR/NDCG@{5,20}, improvement over benchmark)

bf16 emulation (``cfg['bf16']``; the checker of the HIP path's bf16 mode, not a restatement of the
reference): every product the bf16 mode runs on bf16 MFMA operands rounds the same operands at the same
points — the projections (rgemm / wgemm: bf16(x)·bf16(W)ᵀ forward, bf16(dy)·bf16(W) and bf16(dy)ᵀ·bf16(x)
backward, fp32 accumulate, bias sums fp32), the bilinear U = bf16(X2)·bf16(W)ᵀ, and the classifier heads
(ce.hip: logits over bf16(H)·bf16(W)ᵀ, the target and pad logits exact fp32, the softmax parts of dH / dW
over bf16 operands and bf16(softmax·w), the one-hot parts exact).  Attention, LayerNorm, embedding and GCN
stay fp32 in both.

Dropout: the reference draws torch-CPU masks that no GPU RNG can reproduce, so
parity against the reference uses p = 0.  For p > 0 the GPU kernels use a
counter-based hash mask; :func:`keep_mask` restates that hash so the oracle
and the HIP path drop exactly the same elements.
"""
from __future__ import annotations

import math

import numpy as np
import torch

MASK64 = (1 << 64) - 1


# ----------------------------------------------------------------------------- dropout hash
def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def dropout_keys(seed: int, step: int, site: int) -> tuple[int, int]:
    x = _splitmix64((seed & MASK64) ^ _splitmix64((step * 0x100000001B3 + site) & MASK64))
    return x & 0xFFFFFFFF, x >> 32


def _lowbias32(h: np.ndarray) -> np.ndarray:
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x7FEB352D)
    h ^= h >> np.uint32(15)
    h *= np.uint32(0x846CA68B)
    h ^= h >> np.uint32(16)
    return h


def keep_mask(idx: np.ndarray, keys: tuple[int, int], p: float) -> np.ndarray:
    """Bernoulli(1-p) keep decision for flat element indices ``idx`` (int64): one 32-bit hash per pair of
    elements q = idx >> 1, a 16-bit half per element, threshold floor(p·2^16) (c2dsr_amd/csrc/common.h)."""
    if p <= 0.0:
        return np.ones(idx.shape, dtype=bool)
    idx = idx.astype(np.uint64)
    q = idx >> np.uint64(1)
    with np.errstate(over='ignore'):
        h = _lowbias32((q & np.uint64(0xFFFFFFFF)).astype(np.uint32) ^ np.uint32(keys[0]))
        h = _lowbias32(h ^ (q >> np.uint64(32)).astype(np.uint32) ^ np.uint32(keys[1]))
    half = (h >> (np.uint32(16) * (idx & np.uint64(1)).astype(np.uint32))) & np.uint32(0xFFFF)
    thr = max(1, min(0xFFFF, int(math.floor(p * 65536.0))))
    return half >= np.uint32(thr)


# site ids (must match c2dsr_amd/dropout.py)
def site_gcn(table: int, layer: int) -> int:
    return 0x100 + table * 16 + layer


def site_enc(pass_id: int, layer: int, kind: int) -> int:
    # kind: 0 input, 1 attn probs, 2 sa out, 3 ff mid, 4 ff out
    return 0x1000 + pass_id * 256 + (0 if kind == 0 else 1 + layer * 8 + (kind - 1))


class Dropper:
    """Produces fp32 multiplicative dropout masks for a given (seed, step)."""

    def __init__(self, p_gnn: float, p_attn: float, seed: int = 0, step: int = 0, row_offset: int = 0):
        self.p_gnn, self.p_attn, self.seed, self.step = p_gnn, p_attn, seed, step
        self.row_offset = row_offset  # global batch-row offset (data parallel)

    def mask(self, shape, site: int, p: float, row_dim_prod: int | None = None) -> torch.Tensor | None:
        if p <= 0.0:
            return None
        n = int(np.prod(shape))
        base = 0
        if row_dim_prod is not None:
            base = self.row_offset * row_dim_prod
        idx = np.arange(n, dtype=np.int64) + base
        keep = keep_mask(idx, dropout_keys(self.seed, self.step, site), p)
        return torch.from_numpy(keep.reshape(shape).astype(np.float32) / np.float32(1.0 - p))


# ----------------------------------------------------------------------------- bf16 emulation
def _b(x):
    """round to bf16 (RNE) and back"""
    return x.to(torch.bfloat16).to(x.dtype)


class B16Linear(torch.autograd.Function):
    """x·Wᵀ on bf16-rounded operands with fp32 accumulation, and the backward products on bf16-rounded
    operands too (the bf16 mode's rg / wg kernels, csrc/rgemm.hip)."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return _b(x) @ _b(W).T

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        gb = _b(g)
        N, K = W.shape
        return gb @ _b(W), gb.reshape(-1, N).T @ _b(x).reshape(-1, K)


def linear(x, W, b, cfg):
    """nn.Linear: plain fp32, or the bf16 mode's products (cfg['bf16'])."""
    y = B16Linear.apply(x, W) if cfg.get('bf16') else x @ W.T
    return y + b if b is not None else y


class B16CERows(torch.autograd.Function):
    """Per-row cross-entropy terms of one stacked head in the bf16 mode (csrc/ce.hip): lse over the logits
    bf16(H)·bf16(W)ᵀ + b and the fp32 pad logit, minus the target logit taken in fp32 (0 on ignored rows).
    Backward with row weights g: dH = bf16(softmax·g)[:, :n]·bf16(W) − g·W[t], dW = bf16(softmax·g)ᵀ·bf16(H)
    − Σ g·H (one-hot parts exact), db and the pad logit's gradient from the fp32 softmax."""

    @staticmethod
    def forward(ctx, H, W, b, pl, t, ignore):
        n = W.shape[0]
        full = torch.cat([_b(H) @ _b(W).T + b, pl[:, None]], 1)
        lse = torch.logsumexp(full, 1)
        valid = t != ignore
        tc = torch.clamp(t, max=n - 1)
        s_t = torch.where(t < n, (H * W[tc]).sum(-1) + b[tc], pl)
        ctx.save_for_backward(H, W, torch.softmax(full, 1), t, valid)
        return torch.where(valid, lse - s_t, torch.zeros_like(lse))

    @staticmethod
    def backward(ctx, g):
        H, W, Pm, t, valid = ctx.saved_tensors
        n = W.shape[0]
        rw = torch.where(valid, g, torch.zeros_like(g))
        Ps = Pm * rw[:, None]
        on = valid & (t < n)
        tc = torch.clamp(t, max=n - 1)
        oh = torch.zeros(H.shape[0], n, dtype=H.dtype, device=H.device)
        oh[on, tc[on]] = rw[on]
        dH = _b(Ps[:, :n]) @ _b(W) - oh @ W
        dW = _b(Ps[:, :n]).T @ _b(H) - oh.T @ H
        db = Ps[:, :n].sum(0) - oh.sum(0)
        return dH, dW, db, Ps[:, n], None, None


# ----------------------------------------------------------------------------- model pieces
def spmm_coo(row: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n: int, h: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(n, h.shape[1], dtype=h.dtype)
    return out.index_add(0, row, val[:, None] * h[col])


def gcn(E, graph, n_gnn, p, dropper: Dropper, table: int):
    """models/encoders.py:42-48."""
    row, col, val = graph
    hs = [E]
    h = E
    for k in range(n_gnn):
        m = dropper.mask(tuple(h.shape), site_gcn(table, k), p)
        if m is not None:
            h = h * m
        h = spmm_coo(row, col, val, E.shape[0], h)
        hs.append(h)
    return torch.stack(hs, 1).mean(1)


def layer_norm(x, w, b, eps=1e-8):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def attention(x, P, pre, seq, idx_pad, n_head, p, dropper, pass_id, layer, cfg=None):
    """nn.MultiheadAttention → F.multi_head_attention_forward → SDPA (math), with the
    causal float mask + inverted bool kpm merged additively (functional.py mask merge)."""
    cfg = cfg or {}
    B, L, d = x.shape
    dh = d // n_head
    qkv = linear(x, P[pre + 'self_attn.in_proj_weight'], P[pre + 'self_attn.in_proj_bias'], cfg)
    q, k, v = qkv.split(d, dim=-1)
    q = q.reshape(B, L, n_head, dh).transpose(1, 2)
    k = k.reshape(B, L, n_head, dh).transpose(1, 2)
    v = v.reshape(B, L, n_head, dh).transpose(1, 2)
    causal = torch.triu(torch.ones(L, L, dtype=torch.bool), 1)
    kpm = seq != idx_pad  # True ⇒ masked (inverted, Q1)
    masked = causal[None, None] | kpm[:, None, None, :]
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    s = s.masked_fill(masked, float('-inf'))
    row_ok = (~masked).any(-1, keepdim=True)
    s = torch.where(row_ok, s, torch.zeros_like(s))
    a = torch.softmax(s, -1) * row_ok  # fully masked rows → 0 (Q2)
    m = dropper.mask((B, n_head, L, L), site_enc(pass_id, layer, 1), p, row_dim_prod=n_head * L * L)
    if m is not None:
        a = a * m
    o = (a @ v).transpose(1, 2).reshape(B, L, d)
    out = linear(o, P[pre + 'self_attn.out_proj.weight'], P[pre + 'self_attn.out_proj.bias'], cfg)
    m = dropper.mask((B, L, d), site_enc(pass_id, layer, 2), p, row_dim_prod=L * d)
    return out * m if m is not None else out


def feed_forward(x, P, pre, p, dropper, pass_id, layer, cfg=None):
    cfg = cfg or {}
    B, L, d = x.shape
    f = torch.relu(linear(x, P[pre + 'linear1.weight'], P[pre + 'linear1.bias'], cfg))
    m = dropper.mask(tuple(f.shape), site_enc(pass_id, layer, 3), p, row_dim_prod=L * f.shape[-1])
    if m is not None:
        f = f * m
    out = linear(f, P[pre + 'linear2.weight'], P[pre + 'linear2.bias'], cfg)
    m = dropper.mask((B, L, d), site_enc(pass_id, layer, 4), p, row_dim_prod=L * d)
    return out * m if m is not None else out


def self_attention(P, mod, seq, x, pos, cfg, dropper, pass_id):
    """models/encoders.py:29-33 (+ TransformerEncoder / TransformerEncoderLayer)."""
    B, L, d = x.shape
    p = cfg['dropout_attn']
    x = x + P[mod + '.pos_emb.weight'][pos]
    m = dropper.mask((B, L, d), site_enc(pass_id, 0, 0), p, row_dim_prod=L * d)
    if m is not None:
        x = x * m
    for l in range(cfg['n_attn']):
        pre = f'{mod}.encoder.layers.{l}.'
        if cfg['norm_first']:
            x = x + attention(layer_norm(x, P[pre + 'norm1.weight'], P[pre + 'norm1.bias']), P, pre, seq,
                              cfg['idx_pad'], cfg['n_head'], p, dropper, pass_id, l, cfg)
            x = x + feed_forward(layer_norm(x, P[pre + 'norm2.weight'], P[pre + 'norm2.bias']), P, pre, p,
                                 dropper, pass_id, l, cfg)
        else:
            x = layer_norm(x + attention(x, P, pre, seq, cfg['idx_pad'], cfg['n_head'], p, dropper, pass_id, l,
                                         cfg),
                           P[pre + 'norm1.weight'], P[pre + 'norm1.bias'])
            x = layer_norm(x + feed_forward(x, P, pre, p, dropper, pass_id, l, cfg),
                           P[pre + 'norm2.weight'], P[pre + 'norm2.bias'])
    return layer_norm(x, P[mod + '.encoder.norm.weight'], P[mod + '.encoder.norm.bias'])


def embed_names(cfg):
    if cfg['shared_item_embed']:
        return 'embed_i.weight', 'embed_i.weight', 'embed_i.weight'
    return 'embed_i.weight', 'embed_i_a.weight', 'embed_i_b.weight'


def convolve_graph(P, graphs, cfg, dropper):
    """models/C2DSR.py:59-62."""
    es, ea, eb = embed_names(cfg)
    p = cfg['dropout_gnn']
    hs = gcn(P[es], graphs['share'], cfg['n_gnn'], p, dropper, 0)
    ha = gcn(P[ea], graphs['specific'], cfg['n_gnn'], p, dropper, 1)
    hb = gcn(P[eb], graphs['specific'], cfg['n_gnn'], p, dropper, 2)
    return hs, ha, hb


def encode(P, H, ename, mod, seq, pos, cfg, dropper, pass_id):
    scale = cfg['d_latent'] ** 0.5
    E = P[ename]
    # nn.Embedding(padding_idx=pad): the pad row is read but gets no gradient from the lookup
    e = torch.where((seq == cfg['idx_pad'])[..., None], E[seq].detach(), E[seq])
    x = (H[seq] + e) * scale
    return self_attention(P, mod, seq, x, pos, cfg, dropper, pass_id)


def bilinear(x1, x2, W, b, cfg=None):
    if cfg is not None and cfg.get('bf16'):  # U = bf16(x2)·bf16(W)ᵀ (rgemm), s = x1·U in fp32
        out = (x1 * B16Linear.apply(x2, W[0])).sum(-1, keepdim=True)
    else:
        out = torch.einsum('bi,oij,bj->bo', x1, W, x2)
    return out + b if b is not None else out


def bce_logits(s, y, denom=None):
    v = torch.clamp(s, min=0) - s * y + torch.log1p(torch.exp(-s.abs()))
    return v.mean() if denom is None else v.sum() / denom


def cross_entropy(logits, tgt, ignore, denom=None):
    valid = tgt != ignore
    if hasattr(logits, 'rows'):  # bf16 emulation: per-row terms from B16CERows
        return logits.rows.sum() / (valid.sum() if denom is None else denom)
    lse = torch.logsumexp(logits, -1)
    t = torch.where(valid, tgt, torch.zeros_like(tgt))
    picked = logits.gather(1, t[:, None])[:, 0]
    return ((lse - picked) * valid).sum() / (valid.sum() if denom is None else denom)


def loss_counts(batch, cfg):
    """Local counts the loss normalises by: B and the valid targets of the four heads (trainer.py:131-154)."""
    gt_sa, gt_sb, gt_a, gt_b = batch[6], batch[7], batch[8], batch[9]
    n_a, n_b, R = cfg['n_item_a'], cfg['n_item_b'], cfg['len_rec']
    return torch.tensor([gt_sa.shape[0], (gt_sa[:, -R:] != n_a).sum(), (gt_sb[:, -R:] != n_b).sum(),
                         (gt_a[:, -R:] != n_a).sum(), (gt_b[:, -R:] != n_b).sum()], dtype=torch.float64)


def train_forward(P, graphs, batch, cfg, dropper, counts=None):
    """trainer.py:91-156 (+ C2DSR.forward / forward_share).  Returns dict of tensors.

    ``counts`` (data parallelism): the GLOBAL [B, #valid_sa, #valid_sb, #valid_a,
    #valid_b] of the whole batch this rank holds a slice of.  Every mean then divides the local sum by
    the global count, so the per-rank losses (and gradients) sum over ranks to the single-device ones."""
    (seq, seq_a, seq_b, pos, pos_a, pos_b, gt_sa, gt_sb, gt_a, gt_b, gm_a, gm_b, neg_a, neg_b) = batch
    es, ea, eb = embed_names(cfg)
    n_a, n_b, R = cfg['n_item_a'], cfg['n_item_b'], cfg['len_rec']
    B = seq.shape[0]
    out = {}
    hs_t, ha_t, hb_t = convolve_graph(P, graphs, cfg, dropper)
    out['hi_share'], out['hi_a'], out['hi_b'] = hs_t, ha_t, hb_t
    h_share = encode(P, hs_t, es, 'attn_share', seq, pos, cfg, dropper, 0)
    hx = encode(P, ha_t, ea, 'attn_a', seq_a, pos_a, cfg, dropper, 1)
    hy = encode(P, hb_t, eb, 'attn_b', seq_b, pos_b, cfg, dropper, 2)
    h_neg_a = encode(P, hs_t, es, 'attn_share', neg_a, pos, cfg, dropper, 3)
    h_neg_b = encode(P, hs_t, es, 'attn_share', neg_b, pos, cfg, dropper, 4)
    out.update(h_share=h_share, hx=hx, hy=hy, h_neg_a=h_neg_a, h_neg_b=h_neg_b)

    out.update(loss_head(P, h_share, hx, hy, h_neg_a, h_neg_b, batch, cfg, counts))
    return out


def loss_head(P, h_share, hx, hy, h_neg_a, h_neg_b, batch, cfg, counts=None):
    """trainer.py:101-156: pooling (cal_mask), the bilinear discriminators + BCE and the four classifier
    heads + CE, from the five encoder outputs.  Device-agnostic (tests also run it on cuda tensors as the
    fp32 checker of the full-size bf16 head)."""
    (seq, _, _, _, _, _, gt_sa, gt_sb, gt_a, gt_b, gm_a, gm_b, _, _) = batch
    n_a, n_b, R = cfg['n_item_a'], cfg['n_item_b'], cfg['len_rec']
    B = seq.shape[0]
    out = {}
    wa = (gm_a.float() / gm_a.float().sum(-1, keepdim=True))[..., None]
    wb = (gm_b.float() / gm_b.float().sum(-1, keepdim=True))[..., None]
    hx_mean = (hx * wa).sum(1)
    hy_mean = (hy * wb).sum(1)
    Da_b = P.get('D_a.bias')
    Db_b = P.get('D_b.bias')
    sim_a_pos = bilinear(hx_mean, (h_share * wb).sum(1), P['D_a.weight'], Da_b, cfg)
    sim_a_neg = bilinear(hx_mean, (h_neg_a * wa).sum(1), P['D_a.weight'], Da_b, cfg)
    sim_b_pos = bilinear(hy_mean, (h_share * wa).sum(1), P['D_b.weight'], Db_b, cfg)
    sim_b_neg = bilinear(hy_mean, (h_neg_b * wb).sum(1), P['D_b.weight'], Db_b, cfg)
    out['sim_a'] = torch.stack([sim_a_pos, sim_a_neg])
    out['sim_b'] = torch.stack([sim_b_pos, sim_b_neg])
    one = torch.ones(B, 1, device=hx.device)
    zero = torch.zeros(B, 1, device=hx.device)
    cB = None if counts is None else float(counts[0])
    loss_mi = bce_logits(sim_a_pos, one, cB) + bce_logits(sim_a_neg, zero, cB) + \
        bce_logits(sim_b_pos, one, cB) + bce_logits(sim_b_neg, zero, cB)

    hs_r, ha_r, hb_r = h_share[:, -R:], hx[:, -R:], hy[:, -R:]

    Wa, ba, Wb, bb = P['classifier_a.weight'], P['classifier_a.bias'], P['classifier_b.weight'], P['classifier_b.bias']
    t_sa, t_sb = gt_sa[:, -R:].reshape(-1), gt_sb[:, -R:].reshape(-1)
    t_a, t_b = gt_a[:, -R:].reshape(-1), gt_b[:, -R:].reshape(-1)

    def pad_logit(hpad):
        return hpad @ P['classifier_pad.weight'].T + P['classifier_pad.bias']

    if cfg.get('bf16'):  # the fused bf16 heads (csrc/ce.hip): per-row terms, means taken below
        d = h_share.shape[-1]

        class _Rows:
            def __init__(self, h, W, bias, hpad, t, ignore):
                self.rows = B16CERows.apply(h.reshape(-1, d), W, bias, pad_logit(hpad).reshape(-1), t, ignore)

        s_sa = _Rows(hs_r, Wa, ba, hs_r, t_sa, n_a)
        s_sb = _Rows(hs_r, Wb, bb, hs_r, t_sb, n_b)
        s_a = _Rows(hs_r + ha_r, Wa, ba, ha_r, t_a, n_a)
        s_b = _Rows(hs_r + hb_r, Wb, bb, hb_r, t_b, n_b)
    else:
        def head(h, W, bias, hpad):
            return torch.cat([h @ W.T + bias, pad_logit(hpad)], -1)

        s_sa = head(hs_r, Wa, ba, hs_r).reshape(-1, n_a + 1)
        s_sb = head(hs_r, Wb, bb, hs_r).reshape(-1, n_b + 1)
        s_a = head(hs_r + ha_r, Wa, ba, ha_r).reshape(-1, n_a + 1)
        s_b = head(hs_r + hb_r, Wb, bb, hb_r).reshape(-1, n_b + 1)
    if counts is None:
        l_sa = cross_entropy(s_sa, t_sa, n_a)
        l_sb = cross_entropy(s_sb, t_sb, n_b)
        loss_share = l_sa * (t_sa != n_a).sum() / (R * B) + l_sb * (t_sb != n_b).sum() / (R * B)
        l_a = cross_entropy(s_a, t_a, n_a)
        l_b = cross_entropy(s_b, t_b, n_b)
    else:
        c = [float(x) for x in counts]
        l_sa = cross_entropy(s_sa, t_sa, n_a, c[1])
        l_sb = cross_entropy(s_sb, t_sb, n_b, c[2])
        loss_share = l_sa * c[1] / (R * c[0]) + l_sb * c[2] / (R * c[0])
        l_a = cross_entropy(s_a, t_a, n_a, c[3])
        l_b = cross_entropy(s_b, t_b, n_b, c[4])
    loss_rec = loss_share + l_a + l_b
    lam = cfg['lambda_loss']
    loss = lam * loss_rec + (1 - lam) * loss_mi
    out.update(loss=loss, loss_rec=loss_rec, loss_mi=loss_mi, l_sa=l_sa, l_sb=l_sb, l_a=l_a, l_b=l_b)
    return out


# ----------------------------------------------------------------------------- optimizer
class AdamWAmsgrad:
    """torch.optim.AdamW(amsgrad=True) single-tensor update (trainer.py:21-22)."""

    def __init__(self, lr=1e-3, wd=5e-4, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, wd, betas[0], betas[1], eps
        self.state = {}

    def step(self, params: dict, grads: dict):
        for n, g in grads.items():
            if g is None:
                continue
            p = params[n]
            st = self.state.get(n)
            if st is None:
                st = self.state[n] = dict(step=0, m=torch.zeros_like(p), v=torch.zeros_like(p),
                                          vmax=torch.zeros_like(p))
            st['step'] += 1
            t = st['step']
            p.mul_(1 - self.lr * self.wd)
            st['m'].lerp_(g, 1 - self.b1)
            st['v'].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** t
            bc2 = 1 - self.b2 ** t
            torch.maximum(st['vmax'], st['v'], out=st['vmax'])
            denom = (st['vmax'].sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(st['m'], denom, value=-(self.lr / bc1))


def trainable_names(names, cfg):
    """Parameters that ever receive a grad (the encoder_layer template never does, Q15)."""
    skip = {'embed_i_a.weight', 'embed_i_b.weight'} if cfg['shared_item_embed'] else set()
    return [n for n in names if '.encoder_layer.' not in n and (n != 'D_a.bias' or cfg['d_bias'])
            and (n != 'D_b.bias' or cfg['d_bias']) and n not in skip]


class OracleTrainer:
    """Step driver mirroring Trainer.run_epoch's per-batch body (trainer.py:47-53) with
    zero_grad once (Q3)."""

    def __init__(self, params: dict, graphs, cfg, seed=0, lr=1e-3, wd=5e-4):
        self.cfg = cfg
        self.P = {k: v.clone().float().requires_grad_(False) for k, v in params.items()}
        self.names = trainable_names(list(self.P.keys()), cfg)
        self.grads = {n: None for n in self.names}
        self.graphs = graphs
        self.opt = AdamWAmsgrad(lr=lr, wd=wd)
        self.seed = seed
        self.step_no = 0

    def zero_grad(self):
        self.grads = {n: None for n in self.names}

    def train_batch(self, batch, row_offset=0, optimizer=True, counts=None):
        for n in self.names:
            self.P[n].requires_grad_(True)
        dr = Dropper(self.cfg['dropout_gnn'], self.cfg['dropout_attn'], self.seed, self.step_no, row_offset)
        out = train_forward(self.P, self.graphs, batch, self.cfg, dr, counts)
        gs = torch.autograd.grad(out['loss'], [self.P[n] for n in self.names], allow_unused=True)
        for n, g in zip(self.names, gs):
            if g is None:
                continue
            self.grads[n] = g.clone() if self.grads[n] is None else self.grads[n] + g
        for n in self.names:
            self.P[n].requires_grad_(False)
        if optimizer:
            with torch.no_grad():
                self.opt.step(self.P, self.grads)
        self.step_no += 1
        return {k: v.detach() for k, v in out.items()}


def cfg_from_args(a) -> dict:
    return dict(d_latent=a.d_latent, n_item_a=a.n_item_a, n_item_b=a.n_item_b, idx_pad=a.idx_pad,
                len_rec=a.len_rec, lambda_loss=a.lambda_loss, n_gnn=a.n_gnn, n_attn=a.n_attn, n_head=a.n_head,
                norm_first=a.norm_first, d_bias=a.d_bias, shared_item_embed=a.shared_item_embed,
                dropout_gnn=a.dropout_gnn, dropout_attn=a.dropout_attn)


# ----------------------------------------------------------------------------- evaluation (§8 f1)
def evaluate_batch(P, graphs, batch, cfg):
    """trainer.py:162-181 (model.eval(): no dropout; convolve_graph first as in run_epoch:64).
    Returns (rank_a, rank_b) lists, rows in batch order within each domain."""
    (seq, seq_a, seq_b, pos, pos_a, pos_b, il_a, il_b, xory, gt, neg) = batch
    es, ea, eb = embed_names(cfg)
    cfg0 = dict(cfg, dropout_gnn=0.0, dropout_attn=0.0)
    dr = Dropper(0.0, 0.0)
    with torch.no_grad():
        hs_t, ha_t, hb_t = convolve_graph(P, graphs, cfg0, dr)
        h_share = encode(P, hs_t, es, 'attn_share', seq, pos, cfg0, dr, 0)
        hx = encode(P, ha_t, ea, 'attn_a', seq_a, pos_a, cfg0, dr, 1)
        hy = encode(P, hb_t, eb, 'attn_b', seq_b, pos_b, cfg0, dr, 2)
        ra, rb = [], []
        for i in range(seq.shape[0]):
            if int(xory[i]) == 0:
                q = h_share[i, -1] + hx[i, int(il_a[i])]
                s = P['classifier_a.weight'] @ q + P['classifier_a.bias']
                ra.append(int((s[neg[i]] > s[gt[i]]).sum()) + 1)
            else:
                q = h_share[i, -1] + hy[i, int(il_b[i])]
                s = P['classifier_b.weight'] @ q + P['classifier_b.bias']
                rb.append(int((s[neg[i]] > s[gt[i]]).sum()) + 1)
    return ra, rb


def cal_metrics(ranks):
    """utils/metrics.py:4-19."""
    N = len(ranks)
    v = [0.0] * 6
    for r in ranks:
        if r <= 20:
            v[1] += 1
            v[3] += 1 / r
            v[5] += 1 / np.log2(r + 1)
            if r <= 5:
                v[0] += 1
                v[2] += 1 / r
                v[4] += 1 / np.log2(r + 1)
    return [x / N for x in v]


def cal_score(ranks_a, ranks_b, benchmark):
    """utils/metrics.py:22-31."""
    res = cal_metrics(ranks_a) + cal_metrics(ranks_b)
    sel = [res[0], res[4], res[6], res[10]]
    imp = np.array([x / y - 1 for x, y in zip(sel, benchmark)])
    return [float(np.mean(imp))] + res
