"""BASELINE configs[4] (C5) on the GPU at its shape: 10M + 10M items (a 20,000,001-row table), d = 512,
L = 100 — the two HBM-bound kernels of the bench's C5 roofline line (bench.py run_c5) checked on a table of
the full size, through the product's autograd functions: the GCN forward (models/encoders.py:42-48,
H = (E + A·E)/2) and its backward through Aᵀ (K1), the five embedding gathers (models/C2DSR.py:65-71 +
encoders.py:30, K2) and their deterministic segment-sum backward into the table (direct lookups, pad row
excluded) and into the GCN output (then through Aᵀ).  Every full-size output is compared on sampled rows
against fp64 host computations from the same inputs (a float64 restatement of the same op — the oracle of
this property test); dropout 0.  ~170 GB of device memory."""
import math
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def rel_dev(a, b):
    """rel() of two large device tensors, computed on the device."""
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_c5_gcn_and_embedding_at_20m_rows():
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import ops, synth
    from c2dsr_amd.models.encoders import GCN, StepState
    n_a = n_b = 10_000_000
    d, L, B = 512, 100, 256
    N = n_a + n_b + 1
    pad = N - 1
    items, off = synth.make_flat_sequences(200_000, n_a, n_b, L, seed=1)
    seq_id = np.repeat(np.arange(off.size - 1, dtype=np.int64), np.diff(off))
    same = seq_id[1:] == seq_id[:-1]
    g = GR.normalized_csr(np.stack([items[:-1][same], items[1:][same]], 1), N)
    seqs = [items[off[i]:off[i + 1]].tolist() for i in range(2 * B)]
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, n_a, n_b, L))
    assert rows[0].shape[0] >= B
    hb = [r[:B] for r in rows]
    dg = GR.DeviceGraph(g, DEV)
    b = [torch.from_numpy(r.copy()).to(DEV) for r in hb]
    pass_idx = [(0, 3), (1, 4), (2, 5), (12, 3), (13, 3)]  # (seq, pos) of the five passes
    torch.manual_seed(0)
    E = torch.nn.Parameter(torch.empty(N, d, device=DEV).normal_(0.0, 0.1))
    E.grad = torch.zeros_like(E)
    P = torch.nn.Parameter(torch.empty(L, d, device=DEV).normal_(0.0, 0.1))
    P.grad = torch.zeros_like(P)
    state = StepState(seed=1)
    state.step = 1
    gcn = GCN(SimpleNamespace(dropout_gnn=0.0, n_gnn=1, idx_pad=pad))
    gcn.state = state
    H, tok, sink = gcn.propagate(E, dg)
    scale = math.sqrt(d)
    xs = [ops.EmbedFn.apply(tok, E, P, b[s], b[p], H, scale, 0.0, (0, 0), 0, sink, pad) for s, p in pass_idx]
    gx = torch.empty(B, L, d, device=DEV).normal_(0.0, 1.0)
    # forward checks before the backward (the table is unchanged by it; H is consumed by nothing else)
    rng = np.random.default_rng(0)
    r, c, v = g.coo()
    batch_items = np.unique(np.concatenate([hb[s].reshape(-1) for s, _ in pass_idx]))
    batch_items = batch_items[batch_items != pad]
    has_out = np.flatnonzero(np.diff(g.rowptr) > 0)
    h_rows = np.unique(np.concatenate([rng.choice(batch_items, 300, replace=False), rng.choice(has_out, 300)]))
    sel = np.isin(r, h_rows)
    need = np.unique(np.concatenate([h_rows, c[sel]]))
    Eh = dict(zip(need.tolist(), E.detach()[torch.from_numpy(need).to(DEV)].double().cpu().numpy()))
    Hg = H[torch.from_numpy(h_rows).to(DEV)].double().cpu().numpy()
    ref = np.stack([Eh[i] for i in h_rows.tolist()])
    acc = np.zeros_like(ref)
    pos_of = {i: k for k, i in enumerate(h_rows.tolist())}
    for rr, cc, vv in zip(r[sel], c[sel], v[sel]):
        acc[pos_of[int(rr)]] += float(vv) * Eh[int(cc)]
    assert rel(Hg, (ref + acc) / 2) < 1e-5, 'GCN forward (sampled rows)'
    Ph = P.detach().double().cpu().numpy()
    for k, (s, p) in enumerate(pass_idx):
        rr = rng.choice(B * L, 400, replace=False)
        it = hb[s].reshape(-1)[rr]
        ps = hb[p].reshape(-1)[rr]
        Hi = H[torch.from_numpy(it).to(DEV)].double().cpu().numpy()
        Ei = E.detach()[torch.from_numpy(it).to(DEV)].double().cpu().numpy()
        got = xs[k].detach().reshape(B * L, d)[torch.from_numpy(rr).to(DEV)].double().cpu().numpy()
        assert rel(got, (Hi + Ei) * scale + Ph[ps]) < 1e-5, f'embedding forward, pass {k}'
    torch.autograd.backward(xs, [gx] * len(xs))
    torch.cuda.synchronize()
    # host fp64: S_i = Σ over passes and rows with seq = i of gx (per distinct item of the batch)
    G = gx.double().cpu().numpy().reshape(B * L, d)
    uniq = np.unique(np.concatenate([hb[s].reshape(-1) for s, _ in pass_idx]))
    S = np.zeros((uniq.size, d))
    Pref = np.zeros((L, d))
    for s, p in pass_idx:
        np.add.at(S, np.searchsorted(uniq, hb[s].reshape(-1)), G)
        np.add.at(Pref, hb[p].reshape(-1), G)
    assert rel(P.grad.double().cpu().numpy(), Pref) < 1e-5, 'position-table gradient'
    # E.grad[i] = √d·S_i (direct lookups, i != pad) + (√d·S_i + Σ_j A[j, i]·√d·S_j) / 2 (the lookups of H)
    gt = g.transpose()
    has_in = np.flatnonzero(np.diff(gt.rowptr) > 0)
    e_rows = np.unique(np.concatenate([rng.choice(batch_items, 300, replace=False), rng.choice(has_in, 300),
                                       [pad]]))
    Sd = {int(i): S[k] * scale for k, i in enumerate(uniq.tolist())}
    zero = np.zeros(d)
    want = []
    for i in e_rows.tolist():
        t = Sd.get(i, zero).copy()
        for e in range(gt.rowptr[i], gt.rowptr[i + 1]):
            t += float(gt.val[e]) * Sd.get(int(gt.col[e]), zero)
        w = t / 2
        if i != pad:
            w = w + Sd.get(i, zero)
        want.append(w)
    got = E.grad[torch.from_numpy(e_rows).to(DEV)].double().cpu().numpy()
    assert rel(got, np.stack(want)) < 1e-5, 'table gradient (direct lookups + GCN backward through A^T)'


def test_c5_bf16_table_kernels_match_fp32():
    """The C5 roofline run's bf16-table kernels (c2dsr_gcn_spmm_b16, c2dsr_embed_fwd_b16,
    c2dsr_embed_bwd_planned_b16; SURVEY.md §8(d): "bf16 tables") against the fp32 kernels on the same
    (bf16-representable) inputs, at d = 512, L = 100 on a 2,000,001-row table: the arithmetic is fp32 in both,
    so each bf16 result is the fp32 result rounded once (≤ 2^-8 relative) — the gather, whose inputs are the
    same values, is bit-identical — and the five passes' segment sums into a bf16 G round once per pass."""
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import ops, synth
    from c2dsr_amd._lib import lib, stream
    n_a = n_b = 1_000_000
    d, L, B = 512, 100, 128
    N = n_a + n_b + 1
    pad = N - 1
    items, off = synth.make_flat_sequences(100_000, n_a, n_b, L, seed=2)
    seq_id = np.repeat(np.arange(off.size - 1, dtype=np.int64), np.diff(off))
    same = seq_id[1:] == seq_id[:-1]
    g = GR.normalized_csr(np.stack([items[:-1][same], items[1:][same]], 1), N)
    seqs = [items[off[i]:off[i + 1]].tolist() for i in range(2 * B)]
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, n_a, n_b, L))
    b = [torch.from_numpy(r[:B].copy()).to(DEV) for r in rows]
    dg = GR.DeviceGraph(g, DEV)
    torch.manual_seed(0)
    E16 = torch.empty(N, d, device=DEV, dtype=torch.bfloat16).normal_(0.0, 0.1)
    E32 = E16.float()
    keys, p = (11, 22), 0.2
    H16, H32 = torch.empty_like(E16), torch.empty_like(E32)
    ops.spmm(dg, False, E16, keys, p, 0, 0.5, E16, 0.5, 0.0, -1, 0.0, H16)
    ops.spmm(dg, False, E32, keys, p, 0, 0.5, E32, 0.5, 0.0, -1, 0.0, H32)
    assert rel_dev(H16, H32) < 2 ** -8, 'GCN forward on bf16 tables'
    # same fp32 arithmetic in the same edge order (spmm_pf_kernel on bf16 rows, spmm_nc_kernel on fp32 rows), one
    # RNE rounding at the store: bit-equal to the fp32 result rounded to bf16
    assert torch.equal(H16, H32.to(torch.bfloat16)), 'GCN forward on bf16 tables = fp32 forward rounded once'
    P = torch.empty(L, d, device=DEV).normal_(0.0, 0.1)
    passes = [(b[0], b[3]), (b[1], b[4]), (b[2], b[5]), (b[12], b[3]), (b[13], b[3])]
    Hr = H16.float()
    for k, (seq, pos) in enumerate(passes):
        x16, x32 = torch.empty(B, L, d, device=DEV), torch.empty(B, L, d, device=DEV)
        lib('c2dsr_embed_fwd_b16', seq, pos, B * L, d, H16, E16, P, math.sqrt(d), 5, k, p, 0, x16, N, L, None,
            stream())
        lib('c2dsr_embed_fwd', seq, pos, B * L, d, Hr, E32, None, P, math.sqrt(d), 5, k, p, 0, x32, N, L, None,
            stream())
        assert torch.equal(x16, x32), f'gather on bf16 tables, pass {k}'
    gx = torch.empty(B, L, d, device=DEV).normal_(0.0, 1.0)
    G16, G32 = torch.zeros_like(E16), torch.zeros_like(E32)
    gP16, gP32 = torch.zeros_like(P), torch.zeros_like(P)
    ws_bytes = int(lib.raw('c2dsr_embed_bwd_planned_workspace')(B * L, d))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=DEV)
    plans = ops.IndexPlan.many([(seq, N) for seq, _ in passes] + [(pos, L) for _, pos in passes])
    for k in range(len(passes)):
        sp, pp = plans[k].get(), plans[len(passes) + k].get()
        lib('c2dsr_embed_bwd_planned_b16', sp, pp, B * L, d, gx, 5, k, p, 0, math.sqrt(d), G16, N, gP16, L, ws,
            ws_bytes, stream())
        lib('c2dsr_embed_bwd_planned', sp, pp, B * L, d, gx, 5, k, p, 0, math.sqrt(d), G32, N, gP32, L, None, ws,
            ws_bytes, stream())
    torch.cuda.synchronize()
    assert torch.equal(gP16, gP32), 'position sums (fp32 in both)'
    touched = torch.unique(torch.cat([s.reshape(-1) for s, _ in passes]))
    assert rel_dev(G16[touched], G32[touched]) < 5 * 2 ** -8, 'segment sums into a bf16 table'
    untouched = torch.ones(N, dtype=torch.bool, device=DEV)
    untouched[touched] = False
    assert not G16[untouched].any()
    gE16, gE32 = torch.zeros_like(E16), torch.zeros_like(E32)
    Gr = G16.float()
    ops.spmm(dg, True, G16, keys, p, 1, 0.5, G16, 0.5, 1.0, pad, 1.0, gE16)
    ops.spmm(dg, True, Gr, keys, p, 1, 0.5, Gr, 0.5, 1.0, pad, 1.0, gE32)
    assert rel_dev(gE16, gE32) < 2 ** -8, 'GCN backward on bf16 tables'
    assert torch.equal(gE16, gE32.to(torch.bfloat16)), 'GCN backward on bf16 tables = fp32 backward rounded once'
