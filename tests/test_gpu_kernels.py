"""Per-kernel numerics on the MI355X: each HIP kernel (through the C ABI) against a
plain torch-fp32 CPU computation of the same op.  fp32-MFMA paths: rel 1e-5 (of
max |ref|); bf16-MFMA paths: rel 2e-2; integer/index work: bit-exact."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.fixture(scope='module', autouse=True)
def _lib():
    from c2dsr_amd._lib import lib
    assert torch.cuda.is_available()
    lib.load()
    yield


@pytest.mark.parametrize('ta,tb', [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize('prec,tol', [(0, 1e-5), (1, 2e-2)])
@pytest.mark.parametrize('M,N,K', [(300, 200, 96), (128, 128, 32), (37, 53, 19), (256, 768, 256), (64, 40, 5000)])
def test_gemm(ta, tb, prec, tol, M, N, K):
    from c2dsr_amd.ops import gemm
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + ta * 2 + tb)
    A = torch.randn(K, M, generator=g) if ta else torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) if tb else torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    ref = 0.5 * ((A.T if ta else A) @ (B.T if tb else B)) + 2.0 * C0 + bias
    C = C0.to(DEV)
    gemm(A.to(DEV), B.to(DEV), C, M=M, N=N, K=K, transA=ta, transB=tb, alpha=0.5, beta=2.0, bias=bias.to(DEV),
         precision=prec, split_k=1)
    torch.cuda.synchronize()
    assert rel(C, ref) < tol
    # split-K path (no bias)
    ref2 = (A.T if ta else A) @ (B.T if tb else B) + C0
    C = C0.to(DEV)
    gemm(A.to(DEV), B.to(DEV), C, M=M, N=N, K=K, transA=ta, transB=tb, beta=1.0, precision=prec, split_k=0)
    assert rel(C, ref2) < tol


def test_gemm_relu_dropout_epilogue():
    from c2dsr_amd.ops import gemm
    from oracle.c2dsr_oracle import keep_mask
    M, N, K, p = 200, 64, 48, 0.3
    A, W, b = torch.randn(M, K), torch.randn(N, K), torch.randn(N)
    keys = (123456, 987654)
    C = torch.empty(M, N, device=DEV)
    gemm(A.to(DEV), W.to(DEV), C, M=M, N=N, K=K, transB=1, bias=b.to(DEV), relu_drop=(keys, p, 1000), precision=0)
    idx = (np.arange(M)[:, None] + 1000) * N + np.arange(N)[None, :]
    mk = torch.from_numpy(keep_mask(idx, keys, p).astype(np.float32)) / (1 - p)
    ref = torch.relu(A @ W.T + b) * mk
    assert rel(C, ref) < 1e-5


# d = 512 runs the fp32 one-pass-over-the-edges SpMM (spmm_nc_kernel, both 16-byte slices per lane; the C5 width):
# its dropout element index and split-row (hub) combine are checked here against the oracle
@pytest.mark.parametrize('d,n_gnn,p', [(16, 1, 0.0), (64, 1, 0.25), (256, 2, 0.2), (12, 1, 0.0), (512, 1, 0.2),
                                       (512, 2, 0.3)])
def test_gcn_fwd_bwd_vs_oracle(d, n_gnn, p):
    from c2dsr_amd import ops
    from c2dsr_amd.graph import DeviceGraph, normalized_csr
    from oracle import c2dsr_oracle as O
    rng = np.random.default_rng(d + n_gnn)
    N = 700
    edges = rng.integers(0, N - 1, size=(5000, 2))
    hub_out = np.stack([np.full(900, 3), rng.integers(0, N - 1, 900)], 1)  # row 3: 900 edges (split rows)
    hub_in = np.stack([rng.integers(0, N - 1, 700), np.full(700, 5)], 1)   # col 5: a hub in Aᵀ
    edges = np.concatenate([edges, edges[:300], hub_out, hub_in])  # duplicates (counts > 1)
    g = normalized_csr(edges, N)
    dg = DeviceGraph(g, DEV)
    E = torch.randn(N, d)
    seed, step = 3407, 5
    keys = [O.dropout_keys(seed, step, O.site_gcn(1, k)) for k in range(n_gnn)]
    Ed = E.to(DEV).requires_grad_(True)
    sink = ops.GradSink(N, d, DEV)
    H, tok = ops.GCNFn.apply(Ed, dg, n_gnn, p, keys, N - 1, sink)
    dr = O.Dropper(p, 0.0, seed, step)
    r, c, v = g.coo()
    graph = (torch.from_numpy(r), torch.from_numpy(c), torch.from_numpy(v))
    Er = E.clone().requires_grad_(True)
    Hr = O.gcn(Er, graph, n_gnn, p, dr, 1)
    assert rel(H, Hr) < 1e-5
    # backward: inject a dense grad of H through the sink + direct-lookup term on non-pad rows
    G = torch.randn(N, d)
    sink.buf().copy_(G.to(DEV))
    tok.backward()
    ref = torch.autograd.grad(Hr, Er, G)[0] + G * (torch.arange(N) != N - 1)[:, None]
    assert rel(Ed.grad, ref) < 1e-5


@pytest.mark.parametrize('d,n_items,n_rows,p', [(64, 50, 3000, 0.0), (256, 40000, 20000, 0.2), (16, 7, 513, 0.1)])
def test_embed_fwd_bwd_deterministic(d, n_items, n_rows, p):
    from c2dsr_amd._lib import lib, stream
    from oracle.c2dsr_oracle import keep_mask
    rng = np.random.default_rng(d)
    L = 10
    B = n_rows // L
    n_rows = B * L
    # heavy duplication incl. a dominant "pad" id
    seq = rng.integers(0, n_items, size=n_rows)
    seq[rng.random(n_rows) < 0.4] = n_items - 1
    pos = rng.integers(0, L, size=n_rows)
    H, E, P = torch.randn(n_items, d), torch.randn(n_items, d), torch.randn(L, d)
    keys = (11, 22)
    scale = math.sqrt(d)
    X = torch.empty(n_rows, d, device=DEV)
    sd, pd = torch.from_numpy(seq).to(DEV), torch.from_numpy(pos).to(DEV)
    lib('c2dsr_embed_fwd', sd, pd, n_rows, d, H.to(DEV), E.to(DEV), None, P.to(DEV), scale, keys[0], keys[1], p, 77,
        X, n_items, L, None, stream())
    idx = (np.arange(n_rows)[:, None] + 77) * d + np.arange(d)[None, :]
    mk = torch.from_numpy(keep_mask(idx, keys, p).astype(np.float32)) / (1 - p)
    ref = ((H[seq] + E[seq]) * scale + P[pos]) * mk
    assert rel(X, ref) < 1e-6
    gX = torch.randn(n_rows, d)
    outs = []
    for _ in range(2):
        G = torch.zeros(n_items, d, device=DEV)
        gP = torch.zeros(L, d, device=DEV)
        ws_b = lib.raw('c2dsr_embed_bwd_workspace')(n_rows, d)
        ws = torch.empty(ws_b, dtype=torch.uint8, device=DEV)
        lib('c2dsr_embed_bwd', sd, pd, n_rows, d, gX.to(DEV), keys[0], keys[1], p, 77, scale, G, n_items, gP, L, None,
            ws, ws_b, stream())
        outs.append((G.cpu(), gP.cpu()))
    g = gX * mk
    Gr = torch.zeros(n_items, d, dtype=torch.float64).index_add_(0, torch.from_numpy(seq), (g * scale).double())
    Pr = torch.zeros(L, d, dtype=torch.float64).index_add_(0, torch.from_numpy(pos), g.double())
    assert rel(outs[0][0], Gr) < 1e-5 and rel(outs[0][1], Pr) < 1e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])  # bitwise reproducible
    # prebuilt sort plans (side-stream path of ops.EmbedFn): same segment sums, bit for bit
    from c2dsr_amd.ops import IndexPlan
    sp, pp = IndexPlan(sd, n_items), IndexPlan(pd, L)
    G = torch.full((n_items, d), 0.0, device=DEV)
    gP = torch.zeros(L, d, device=DEV)
    gXin = torch.empty(n_rows, d, device=DEV)
    ws_b = lib.raw('c2dsr_embed_bwd_planned_workspace')(n_rows, d)
    ws = torch.empty(ws_b, dtype=torch.uint8, device=DEV)
    lib('c2dsr_embed_bwd_planned', sp.get(), pp.get(), n_rows, d, gX.to(DEV), keys[0], keys[1], p, 77, scale, G,
        n_items, gP, L, gXin, ws, ws_b, stream())
    off = lib.raw('c2dsr_plan_err_offset')(n_rows)
    assert int(sp.get()[off:off + 4].view(torch.int32).item()) == 0
    # a plan of other indices (keys past the output rows) is skipped and flagged, never followed
    bad = IndexPlan(torch.full((n_rows,), n_items + 5, dtype=torch.int64, device=DEV), n_items + 6)
    G2 = torch.zeros(n_items, d, device=DEV)
    lib('c2dsr_embed_bwd_planned', bad.get(), None, n_rows, d, gX.to(DEV), keys[0], keys[1], p, 77, scale, G2,
        n_items, None, L, None, ws, ws_b, stream())
    assert int(bad.get()[off:off + 4].view(torch.int32).item()) != 0 and float(G2.abs().sum()) == 0.0
    assert torch.equal(G.cpu(), outs[0][0]) and torch.equal(gP.cpu(), outs[0][1])
    assert rel(gXin, gX * mk) < 1e-6
    # the plan itself: keys ascending, rows ascending within a key (stable)
    pl = sp.get().cpu()
    nb = (n_rows * 4 + 255) // 256 * 256
    kk = pl[:n_rows * 4].view(torch.int32).numpy()
    vv = pl[nb:nb + n_rows * 4].view(torch.int32).numpy()
    order = np.lexsort((np.arange(n_rows), seq))
    assert np.array_equal(kk, seq[order]) and np.array_equal(vv, order)
    # gX given as two compact row sources (the row-subset attention layer, d >= 64): the same sums as on the
    # combined rows
    if d < 64:  # not supported there: refused
        from c2dsr_amd._lib import HipLibError
        with pytest.raises(HipLibError, match='hipError 1'):
            lib('c2dsr_embed_bwd_planned_rows', sp.get(), None, n_rows, d, None, None, None, None, 0, 0, 0.0, 0, 1.0,
                None, n_items, None, L, None, 0, stream())
    else:
        ma, mb = rng.random(n_rows) < 0.4, rng.random(n_rows) < 0.6
        inv_a, inv_b = np.full(n_rows, -1, np.int32), np.full(n_rows, -1, np.int32)
        inv_a[ma], inv_b[mb] = np.arange(ma.sum()), np.arange(mb.sum())
        ga, gb = torch.randn(int(ma.sum()), d, device=DEV), torch.randn(int(mb.sum()), d, device=DEV)
        ia, ib = torch.from_numpy(inv_a).to(DEV), torch.from_numpy(inv_b).to(DEV)
        gfull = torch.empty(n_rows, d, device=DEV)
        lib('c2dsr_combine_rows', ga, ia, gb, ib, n_rows, d, gfull, stream())
        res = []
        for rows in (False, True):
            G3, gP3 = torch.zeros(n_items, d, device=DEV), torch.zeros(L, d, device=DEV)
            if rows:
                lib('c2dsr_embed_bwd_planned_rows', sp.get(), pp.get(), n_rows, d, ga, ia, gb, ib, keys[0], keys[1], p, 77,
                    scale, G3, n_items, gP3, L, ws, ws_b, stream())
            else:
                lib('c2dsr_embed_bwd_planned', sp.get(), pp.get(), n_rows, d, gfull, keys[0], keys[1], p, 77, scale, G3,
                    n_items, gP3, L, None, ws, ws_b, stream())
            res.append((G3, gP3))
        assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def _tail_of_segment(t):
    """A device copy of ``t`` whose storage ENDS where its own hipMalloc segment ends (the caching allocator
    gives requests >= 10 MB, rounded to 2 MB, a segment of their own): a kernel reading past the tensor's
    last element leaves the allocation (regression guard for the round-1 attention fault)."""
    torch.cuda.empty_cache()
    seg = 2 << 20
    nbytes = max(12 << 20, -(-t.numel() * 4 // seg) * seg)
    buf = torch.empty(nbytes // 4, device=DEV, dtype=torch.float32)
    out = buf[buf.numel() - t.numel():].view(t.shape)
    out.copy_(t.to(DEV))
    return out


def _attention_case(B, L, d, H, p, tail=False):
    from c2dsr_amd import ops
    from oracle import c2dsr_oracle as O
    torch.manual_seed(L + d + B)
    pad = 999
    lens = torch.randint(1, L, (B,))
    seq = torch.randint(0, 900, (B, L))
    for b in range(B):  # left padding; position 0 always pad, plus random interior pads
        seq[b, :L - lens[b]] = pad
    seq[torch.rand(B, L) < 0.3] = pad
    seq[:, 0] = pad
    qkv = torch.randn(B, L, 3 * d)
    seed, step = 5, 9
    dr = O.Dropper(0.0, p, seed, step)
    keys = O.dropout_keys(seed, step, O.site_enc(2, 0, 1))
    qd = (_tail_of_segment(qkv) if tail else qkv.to(DEV)).requires_grad_(True)
    out = ops.AttnFn.apply(qd, seq.to(DEV), pad, H, p, keys, 0)
    # the oracle's attention math (oracle/c2dsr_oracle.py:attention) on the given q, k, v
    qr = qkv.clone().requires_grad_(True)
    dh = d // H
    q, k, v = qr.split(d, -1)
    q = q.reshape(B, L, H, dh).transpose(1, 2)
    k = k.reshape(B, L, H, dh).transpose(1, 2)
    v = v.reshape(B, L, H, dh).transpose(1, 2)
    causal = torch.triu(torch.ones(L, L, dtype=torch.bool), 1)
    masked = causal[None, None] | (seq != pad)[:, None, None, :]
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    s = s.masked_fill(masked, float('-inf'))
    ok = (~masked).any(-1, keepdim=True)
    a = torch.softmax(torch.where(ok, s, torch.zeros_like(s)), -1) * ok
    m = dr.mask((B, H, L, L), O.site_enc(2, 0, 1), p, row_dim_prod=H * L * L)
    if m is not None:
        a = a * m
    ref = (a @ v).transpose(1, 2).reshape(B, L, d)
    assert rel(out, ref) < 1e-5
    go = torch.randn(B, L, d)
    out.backward(_tail_of_segment(go) if tail else go.to(DEV))
    ref.backward(go)
    torch.cuda.synchronize()
    assert rel(qd.grad, qr.grad) < 1e-5


@pytest.mark.parametrize('L,d,H,p', [(8, 16, 1, 0.0), (8, 16, 2, 0.0), (50, 256, 1, 0.2), (30, 64, 2, 0.1),
                                     (100, 128, 1, 0.0), (128, 64, 4, 0.0)])
def test_attention_vs_oracle(L, d, H, p):
    _attention_case(24, L, d, H, p)


# wave path: L <= 64 and d/H % 32 == 0; tiled otherwise.  Short / odd last batches with qkv (and dout)
# ending exactly at the end of their allocation: the round-1 fault was a wave-path buffer descriptor
# reaching past the last sequence (test_train_steps_match_reference[shared], B 8, L 8, d 16).
@pytest.mark.parametrize('B,L,d,H,p', [(8, 8, 16, 1, 0.0), (13, 50, 256, 1, 0.2), (7, 8, 64, 2, 0.0),
                                       (5, 100, 128, 1, 0.1), (1, 50, 256, 1, 0.0), (3, 64, 32, 1, 0.0)])
def test_attention_short_batch_at_allocation_end(B, L, d, H, p):
    _attention_case(B, L, d, H, p, tail=True)


@pytest.mark.parametrize('d', [16, 64, 256, 512])
@pytest.mark.parametrize('p', [0.0, 0.2])
def test_add_layernorm_fwd_bwd(d, p):
    from c2dsr_amd import ops
    from oracle.c2dsr_oracle import keep_mask
    rows = 777
    a, b = torch.randn(rows, d), torch.randn(rows, d)
    w, bias = torch.randn(d), torch.randn(d)
    keys = (5, 6)
    ad, bd = a.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    bsd = bias.to(DEV).requires_grad_(True)
    y = ops.AddLNFn.apply(ad, bd, wd, bsd, p, keys, 10, 1e-8)
    idx = (np.arange(rows)[:, None] + 10) * d + np.arange(d)[None, :]
    mk = torch.from_numpy(keep_mask(idx, keys, p).astype(np.float32)) / (1 - p)
    ar, br, wr, bbr = [t.clone().requires_grad_(True) for t in (a, b, w, bias)]
    x = ar + br * mk
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    ref = (x - mu) / torch.sqrt(var + 1e-8) * wr + bbr
    assert rel(y, ref) < 1e-5
    gy = torch.randn(rows, d)
    y.backward(gy.to(DEV))
    ref.backward(gy)
    for got, want in ((ad.grad, ar.grad), (bd.grad, br.grad), (wd.grad, wr.grad), (bsd.grad, bbr.grad)):
        assert rel(got, want) < 2e-5


def test_adamw_kernel_vs_oracle():
    from c2dsr_amd._lib import lib, stream
    from oracle.c2dsr_oracle import AdamWAmsgrad
    n = 10_000
    p = torch.randn(n)
    opt = AdamWAmsgrad(lr=1e-3, wd=5e-4)
    P = {'w': p.clone()}
    bufs = [p.clone().to(DEV)] + [torch.zeros(n, device=DEV) for _ in range(5)]
    pd, fresh, accum, m, v, vmax = bufs
    acc_ref = torch.zeros(n)
    for step in range(1, 4):
        g = torch.randn(n)
        acc_ref += g
        fresh.copy_(g.to(DEV))
        lib('c2dsr_adamw', pd, fresh, accum, m, v, vmax, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, step, None, stream())
        opt.step(P, {'w': acc_ref.clone()})
        assert rel(pd, P['w']) < 1e-6
        assert float(fresh.abs().max()) == 0.0
        assert rel(accum, acc_ref) < 1e-7


def test_adamw_direct_accumulation_vs_oracle():
    """One device: the backward accumulates into the epoch accumulator itself (fresh == accum, FlatStore
    direct); the kernel only reads it (36 B/param) and the update equals the oracle's."""
    from c2dsr_amd._lib import lib, stream
    from oracle.c2dsr_oracle import AdamWAmsgrad
    n = 10_000
    p = torch.randn(n)
    opt = AdamWAmsgrad(lr=1e-3, wd=5e-4)
    P = {'w': p.clone()}
    pd = p.clone().to(DEV)
    acc, m, v, vmax = (torch.zeros(n, device=DEV) for _ in range(4))
    acc_ref = torch.zeros(n)
    for step in range(1, 4):
        g = torch.randn(n)
        acc_ref += g
        acc += g.to(DEV)
        lib('c2dsr_adamw', pd, acc, acc, m, v, vmax, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, step, None, stream())
        opt.step(P, {'w': acc_ref.clone()})
        assert rel(pd, P['w']) < 1e-6
        assert rel(acc, acc_ref) < 1e-6  # read only


def test_transposed_lds_fragment_addressing():
    """ds_read_b64_tr_b16 + swizzled image: the fragment layout the fused CE kernels rely on."""
    from c2dsr_amd._lib import lib, stream
    for rr0, kb0 in ((0, 0), (16, 32), (32, 128), (48, 224)):
        out = torch.zeros(1024, dtype=torch.int16, device=DEV)
        lib('c2dsr_selftest_tr', rr0, kb0, out, stream())
        got = out.cpu().numpy().astype(np.int64)
        for lane in range(64):
            h = lane >> 5
            for j in range(8):
                row = rr0 + 8 * (j >> 2) + 4 * h + (j & 3)
                assert got[lane * 8 + j] == row * 256 + kb0 + (lane & 31), (rr0, kb0, lane, j)
                rrow = rr0 + (lane & 31)
                if rr0 + 31 < 64:
                    assert got[512 + lane * 8 + j] == rrow * 256 + kb0 + 8 * h + j, ('row', rr0, kb0, lane, j)


def _bf16(t):
    return t.to(torch.bfloat16).to(torch.float32)


# the bf16-mode fwd_u / dw pair: ce.hip (32x32x16, 64-row stationary blocks) and ce3.hip's plain-bf16
# instantiation (16x16x32, the kernel the bf16 mode runs for D = 128 / 256) — same arguments, same outputs
CE_B16 = {'ce': ('c2dsr_ce_fused_fwd_u', 'c2dsr_ce_fused_dw'), 'ce3b': ('c2dsr_ce3b_fused_fwd_u', 'c2dsr_ce3b_fused_dw')}


@pytest.mark.parametrize('kern', sorted(CE_B16))
@pytest.mark.parametrize('M,n,D', [(300, 700, 256), (1000, 2100, 128), (64, 65, 256), (777, 4099, 256), (33, 31, 128)])
def test_fused_linear_ce_vs_reference(M, n, D, kern):
    """K5 fused head (bf16 MFMA) vs a float64 CPU computation of the same op on the same bf16-rounded
    operands: lse rel 2e-5; gradients (P' rounded to bf16 for the 2nd product) rel 1e-2 of max."""
    fwd_u, fdw = CE_B16[kern]
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(M + n)
    H = _bf16(torch.randn(M, D, generator=g) * 0.5)
    W = _bf16(torch.randn(n, D, generator=g) * 0.5)
    b = torch.randn(n, generator=g) * 0.1
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n + 1, (M,), generator=g)
    t[:5] = n  # ignored rows
    BR = M // 2
    coef = torch.tensor([0.37, 1.9])
    gs = torch.tensor([1.0])
    lam = 0.7
    s = stream()
    d = lambda x: x.to(DEV)  # noqa: E731
    M_pad = -(-M // 64) * 64
    Hb = torch.zeros(M_pad, D, dtype=torch.bfloat16, device=DEV)  # whole 64-row H tiles: zero rows past M
    Hb[:M] = d(H.to(torch.bfloat16))
    n64 = -(-n // 64) * 64  # the fused kernels read whole 64-row W tiles: zero rows past n
    Wb = torch.zeros(n64, D, dtype=torch.bfloat16, device=DEV)
    Wb[:n] = d(W.to(torch.bfloat16))
    ns, nr = 3, 2
    n_pad = -(-n // 128) * 128 + 64
    bias2 = torch.empty(n_pad, device=DEV)
    lib('c2dsr_ce_bias2', d(b), n, n_pad, bias2, s)
    pm, ps = torch.empty(ns, M, device=DEV), torch.empty(ns, M, device=DEV)
    lse, rows = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    lse2 = torch.empty(M_pad, device=DEV)
    lib('c2dsr_ce_fused_fwd', Hb, Wb, bias2, M, n, D, ns, pm, ps, d(pl), d(t), d(H), d(W), d(b), lse, lse2, rows, s)
    # reference
    lg = torch.cat([H.double() @ W.double().T + b.double(), pl.double()[:, None]], 1)
    lse_r = torch.logsumexp(lg, 1)
    valid = t != n
    rows_r = torch.where(valid, lse_r - lg.gather(1, t[:, None])[:, 0], torch.zeros(M, dtype=torch.float64))
    assert rel(lse, lse_r) < 2e-5
    assert rel(rows, rows_r) < 1e-4
    rw, dpad = torch.empty(M_pad, device=DEV), torch.empty(M, device=DEV)
    t32 = torch.empty(M_pad, device=DEV, dtype=torch.int32)
    crow = torch.empty(M_pad + 64, device=DEV)
    lib('c2dsr_ce_row_weights', d(t), M, M_pad, n, d(coef), BR, d(gs), lam, d(pl), lse, rw, t32, lse2, crow, dpad, s)
    w_r = torch.where(valid, lam * coef[(torch.arange(M) >= BR).long()].double(), torch.zeros(M, dtype=torch.float64))
    P = torch.softmax(lg, 1)
    oh = torch.zeros_like(P)
    oh[torch.arange(M), t] = 1.0
    dl = (P - oh) * w_r[:, None]
    assert rel(rw[:M], w_r) < 1e-6 and rel(dpad, dl[:, n]) < 1e-4
    dH = torch.empty(M, D, device=DEV)
    dHp = torch.empty(ns, M, D, device=DEV)
    lib('c2dsr_ce_fused_dh', Hb, Wb, bias2, M, n, D, ns, crow, dHp, s)
    lib('c2dsr_ce_dh_combine', dHp, ns, M, D, t32, rw, d(W), n, dH, s)
    assert rel(dH, dl[:, :n] @ W.double()) < 1e-2
    # forward with the softmax part of dH accumulated online (lazy max rescale), then dH from its partials
    pm2, ps2 = torch.empty(ns, M, device=DEV), torch.empty(ns, M, device=DEV)
    Up = torch.empty(ns, M, D, device=DEV)
    lse_u, rows_u = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    lse2_u = torch.empty(M_pad, device=DEV)
    lib(fwd_u, Hb, Wb, bias2, M, n, D, ns, pm2, ps2, Up, d(pl), d(t), d(H), d(W), d(b), lse_u, lse2_u, rows_u, s)
    assert rel(lse_u, lse_r) < 2e-5
    assert rel(rows_u, rows_r) < 1e-4
    dHu = torch.empty(M, D, device=DEV)
    lib('c2dsr_ce_dh_from_u', Up, pm2, ns, M, D, lse2_u, t32, rw, d(W), n, dHu, s)
    assert rel(dHu, dl[:, :n] @ W.double()) < 1e-2
    gW = torch.ones(n, D, device=DEV)
    gb = torch.ones(n, device=DEV)
    dWp, dbp = torch.empty(nr, n, D, device=DEV), torch.empty(nr, n, device=DEV)
    lib(fdw, Hb, Wb, bias2, M, n, D, nr, crow, dWp, dbp, s)
    lib('c2dsr_sum_parts', dWp, nr, n * D, 1.0, gW, s)
    lib('c2dsr_sum_parts', dbp, nr, n, 1.0, gb, s)
    wsb = int(lib.raw('c2dsr_ce_onehot_workspace')(M, n, D))
    ws = torch.empty(wsb, device=DEV, dtype=torch.uint8)
    gW0, gb0 = gW.clone(), gb.clone()
    lib('c2dsr_ce_onehot_dw', d(t), M, n, d(H), D, rw, gW, gb, ws, wsb, s)
    assert rel(gW - 1, dl[:, :n].T @ H.double()) < 1e-2
    assert rel(gb - 1, dl[:, :n].sum(0)) < 1e-2
    # the same on a prebuilt target plan: bit for bit
    from c2dsr_amd.ops import IndexPlan
    tp = IndexPlan(d(t), n + 1)
    wsb = int(lib.raw('c2dsr_ce_onehot_planned_workspace')(M, n, D))
    ws = torch.empty(wsb, device=DEV, dtype=torch.uint8)
    lib('c2dsr_ce_onehot_dw_planned', tp.get(), M, n, d(H), D, rw, gW0, gb0, ws, wsb, s)
    assert torch.equal(gW0, gW) and torch.equal(gb0, gb)


@pytest.mark.parametrize('kern', sorted(CE_B16))
@pytest.mark.parametrize('M,n,D,ns', [(200, 1500, 256, 2), (333, 3000, 128, 5), (130, 900, 256, 1)])
def test_fused_ce_online_rescale(M, n, D, ns, kern):
    """c2dsr_ce_fused_fwd_u when the row max keeps rising across column tiles (bias ramp of 60 nats and
    a column-dependent scale: the lazy rescale fires many times, at different tiles for different rows
    of one wave) and when it falls (reversed ramp on half of the rows via their H sign): lse vs float64,
    dH = rw·(softmax·W − W[t]) vs float64."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(M * 7 + n)
    H = _bf16(torch.randn(M, D, generator=g) * 0.3)
    H[1::2, :8] = _bf16(-H[1::2, :8].abs() - 1.0)
    H[0::2, :8] = _bf16(H[0::2, :8].abs() + 1.0)
    W = torch.randn(n, D, generator=g) * 0.2
    W[:, :8] = torch.linspace(-2.0, 2.0, n)[:, None]  # a score ramp rising for even rows, falling for odd rows
    W = _bf16(W)
    b = torch.linspace(0.0, 60.0, n) * (torch.rand(n, generator=g) > 0.5)
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n, (M,), generator=g)
    s = stream()
    d = lambda x: x.to(DEV)  # noqa: E731
    M_pad = -(-M // 64) * 64
    Hb = torch.zeros(M_pad, D, dtype=torch.bfloat16, device=DEV)
    Hb[:M] = d(H.to(torch.bfloat16))
    n64 = -(-n // 64) * 64
    Wb = torch.zeros(n64, D, dtype=torch.bfloat16, device=DEV)
    Wb[:n] = d(W.to(torch.bfloat16))
    n_pad = -(-n // 128) * 128 + 64
    bias2 = torch.empty(n_pad, device=DEV)
    lib('c2dsr_ce_bias2', d(b), n, n_pad, bias2, s)
    pm, ps = torch.empty(ns, M, device=DEV), torch.empty(ns, M, device=DEV)
    Up = torch.empty(ns, M, D, device=DEV)
    lse, rows = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    lse2 = torch.empty(M_pad, device=DEV)
    lib(CE_B16[kern][0], Hb, Wb, bias2, M, n, D, ns, pm, ps, Up, d(pl), d(t), d(H), d(W), d(b), lse, lse2, rows, s)
    lg = torch.cat([H.double() @ W.double().T + b.double(), pl.double()[:, None]], 1)
    lse_r = torch.logsumexp(lg, 1)
    assert rel(lse, lse_r) < 2e-5
    coef, gs, lam = torch.tensor([0.5, 1.5]), torch.tensor([1.0]), 0.7
    rw, dpad = torch.empty(M_pad, device=DEV), torch.empty(M, device=DEV)
    t32 = torch.empty(M_pad, device=DEV, dtype=torch.int32)
    crow = torch.empty(M_pad + 64, device=DEV)
    lib('c2dsr_ce_row_weights', d(t), M, M_pad, n, d(coef), M // 2, d(gs), lam, d(pl), lse, rw, t32, lse2, crow,
        dpad, s)
    dH = torch.empty(M, D, device=DEV)
    lib('c2dsr_ce_dh_from_u', Up, pm, ns, M, D, lse2, t32, rw, d(W), n, dH, s)
    w_r = lam * coef[(torch.arange(M) >= M // 2).long()].double()
    P = torch.softmax(lg, 1)
    oh = torch.zeros_like(P)
    oh[torch.arange(M), t] = 1.0
    ref = ((P - oh) * w_r[:, None])[:, :n] @ W.double()
    assert rel(dH, ref) < 1e-2
    assert torch.isfinite(Up).all()


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize('M,N,K', [(1000, 768, 256), (300, 256, 768), (129, 256, 256), (77, 320, 512)])
def test_rgemm_vs_bf16_rounded_fp32(M, N, K):
    """Row-streaming projection GEMM: exact products of bf16-rounded operands, fp32 sums."""
    from c2dsr_amd.ops import rgemm, rgemm_ok, to_bf16
    assert rgemm_ok(M, N, K)
    g = torch.Generator().manual_seed(M + N + K)
    A, W, C0, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(M, N, generator=g), \
        torch.randn(N, generator=g)
    C = C0.to(DEV)
    rgemm(A.to(DEV), to_bf16(W.to(DEV)), C, M=M, N=N, K=K, alpha=0.5, bias=b.to(DEV))
    ref = 0.5 * (_bf(A).double() @ _bf(W).double().T) + b.double()
    assert rel(C, ref) < 2e-6
    # transposed weight copy (the dx = dy·W product)
    Wt = torch.randn(K, N, generator=g)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), to_bf16(Wt.to(DEV), trans=True), C, M=M, N=N, K=K)
    assert rel(C, _bf(A).double() @ _bf(Wt).double()) < 2e-6


def test_rgemm_relu_dropout_epilogue():
    from c2dsr_amd.ops import rgemm, to_bf16
    from oracle.c2dsr_oracle import keep_mask
    M, N, K, p = 333, 256, 256, 0.3
    A, W, b = torch.randn(M, K), torch.randn(N, K), torch.randn(N)
    keys = (123456, 987654)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), to_bf16(W.to(DEV)), C, M=M, N=N, K=K, bias=b.to(DEV), relu_drop=(keys, p, 1000))
    idx = (np.arange(M)[:, None] + 1000) * N + np.arange(N)[None, :]
    mk = torch.from_numpy(keep_mask(idx, keys, p).astype(np.float32)).double() / (1 - p)
    ref = torch.relu(_bf(A).double() @ _bf(W).double().T + b.double()) * mk
    assert rel(C, ref) < 2e-6


@pytest.mark.parametrize('T,N', [(1000, 256), (4097, 768), (31, 128)])
def test_wgemm_vs_bf16_rounded_fp32(T, N):
    """Projection weight gradient: dW = beta·dW + dYᵀ·X (bf16-rounded operands, fp32 sums)."""
    from c2dsr_amd.ops import wgemm, wgemm_ok
    D = 256
    assert wgemm_ok(T, N, D)
    g = torch.Generator().manual_seed(T + N)
    dY, X, W0 = torch.randn(T, N, generator=g), torch.randn(T, D, generator=g), torch.randn(N, D, generator=g)
    dW = W0.to(DEV)
    wgemm(dY.to(DEV), X.to(DEV), dW, T=T, N=N, D=D, beta=1.0)
    ref = W0.double() + _bf(dY).double().T @ _bf(X).double()
    assert rel(dW, ref) < 1e-5
    dW = torch.full((N, D), 7.0, device=DEV)
    db = torch.full((N,), 3.0, device=DEV)
    wgemm(dY.to(DEV), X.to(DEV), dW, T=T, N=N, D=D, beta=0.0, db=db)
    assert rel(dW, _bf(dY).double().T @ _bf(X).double()) < 1e-5
    assert rel(db, dY.double().sum(0)) < 1e-6  # fp32 column sums of the unrounded dY
    db1 = torch.ones(N, device=DEV)
    wgemm(dY.to(DEV), X.to(DEV), torch.zeros(N, D, device=DEV), T=T, N=N, D=D, beta=1.0, db=db1)
    assert rel(db1, 1.0 + dY.double().sum(0)) < 1e-6
    # deterministic: same bits on a re-run
    dW2 = torch.full((N, D), 7.0, device=DEV)
    wgemm(dY.to(DEV), X.to(DEV), dW2, T=T, N=N, D=D, beta=0.0)
    assert torch.equal(dW, dW2)


@pytest.mark.parametrize('K', [256, 768])
def test_rgemm_aux_epilogues(K):
    """c2dsr_rgemm_aux: in-place accumulate (the residual-gradient sum) and the drop(relu) backward mask,
    against bf16-rounded fp32 products; odd row-tile counts exercise the repeated last tile."""
    from c2dsr_amd.ops import AUX_ACC, AUX_ACC_MAP, AUX_MASK, rgemm, to_bf16
    g = torch.Generator().manual_seed(K)
    M, N = 32 * 37 + 5, 256
    A, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
    Wb = to_bf16(W.to(DEV))
    prod = _bf(A).double() @ _bf(W).double().T
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(DEV)
    rgemm(A.to(DEV), Wb, C, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C)
    assert rel(C, prod + C0.double()) < 2e-6
    src = torch.randn(M, N, generator=g)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), Wb, C, M=M, N=N, K=K, aux_mode=AUX_MASK, aux=src.to(DEV), aux_scale=1.25)
    want = torch.where(src.double() > 0, prod * 1.25, torch.zeros_like(prod))
    assert rel(C, want) < 2e-6
    # AUX_ACC_MAP: aux holds a compacted subset of the rows, read through the row map
    keep = torch.nonzero(torch.rand(M, generator=g) < 0.6).reshape(-1)
    inv = torch.full((M,), -1, dtype=torch.int32)
    inv[keep] = torch.arange(keep.numel(), dtype=torch.int32)
    park = torch.randn(keep.numel(), N, generator=g)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), Wb, C, M=M, N=N, K=K, aux_mode=AUX_ACC_MAP, aux=park.to(DEV), auxmap=inv.to(DEV))
    full = torch.zeros(M, N, dtype=torch.float64)
    full[keep] = park.double()
    assert rel(C, prod + full) < 2e-6


@pytest.mark.parametrize('B,L,R', [(1, 7, 3), (37, 50, 10), (300, 50, 10), (2048, 50, 10)])
def test_need_rows_compaction(B, L, R):
    """c2dsr_need_rows: five sets in one pass (stable, across 1024-row tiles) vs numpy."""
    from c2dsr_amd._lib import lib, stream
    g = np.random.default_rng(B)
    gm_a = (g.random((B, L)) < 0.3).astype(np.int64)
    gm_b = (g.random((B, L)) < 0.2).astype(np.int64)
    codes = (7, 5, 6, 1, 2)
    M, n = B * L, len(codes)
    idx = torch.full((n, M), -7, device=DEV, dtype=torch.int32)
    inv = torch.empty(n, M, device=DEV, dtype=torch.int32)
    cnt = torch.empty(n, device=DEV, dtype=torch.int32)
    off = torch.empty(n, B + 1, device=DEV, dtype=torch.int32)
    ws = torch.empty(lib.raw('c2dsr_compact_workspace')(M, n) // 4 + 1, device=DEV, dtype=torch.int32)
    bits = sum(c << (3 * q) for q, c in enumerate(codes))
    lib('c2dsr_need_rows', torch.from_numpy(gm_a).to(DEV), torch.from_numpy(gm_b).to(DEV), B, L, R, n, bits, idx,
        inv, cnt, off, ws, stream())
    tail = np.broadcast_to(np.arange(L) >= L - R, (B, L)).reshape(-1)
    a, b = gm_a.reshape(-1) != 0, gm_b.reshape(-1) != 0
    for q, c in enumerate(codes):
        need = (a if c & 1 else False) | (b if c & 2 else False) | (tail if c & 4 else False)
        _check_row_set(need, idx[q], inv[q], cnt[q], off[q], B, L)


def _check_row_set(need, idx, inv, cnt, off, B, L):
    M = B * L
    want = np.nonzero(need)[0]
    assert int(cnt) == len(want)
    assert np.array_equal(idx[:len(want)].cpu().numpy(), want)
    winv = np.full(M, -1)
    winv[want] = np.arange(len(want))
    assert np.array_equal(inv.cpu().numpy(), winv)
    woff = np.concatenate([[0], np.cumsum(need.reshape(B, L).sum(1))])
    assert np.array_equal(off.cpu().numpy(), woff)


@pytest.mark.parametrize('B,L', [(1, 7), (37, 50), (2048, 50)])
def test_pad_rows_compaction(B, L):
    """c2dsr_pad_rows: padding rows of five sequences at once, with per-sequence offsets."""
    from c2dsr_amd._lib import lib, stream
    g = np.random.default_rng(B + 1)
    pad = 77
    seqs = g.integers(0, 70, (5, B, L))
    seqs[g.random((5, B, L)) < 0.45] = pad
    seqs[0, :, :L // 2] = pad  # left padding
    seqs[1, 0] = pad           # an all-padding sequence
    seqs[2, -1] = 3            # one without padding
    M, n = B * L, 5
    idx = torch.full((n, M), -7, device=DEV, dtype=torch.int32)
    inv = torch.empty(n, M, device=DEV, dtype=torch.int32)
    cnt = torch.empty(n, device=DEV, dtype=torch.int32)
    off = torch.empty(n, B + 1, device=DEV, dtype=torch.int32)
    ws = torch.empty(lib.raw('c2dsr_compact_workspace')(M, n) // 4 + 1, device=DEV, dtype=torch.int32)
    lib('c2dsr_pad_rows', torch.from_numpy(seqs).to(DEV), pad, B, L, n, idx, inv, cnt, off, ws, stream())
    for q in range(n):
        _check_row_set(seqs[q].reshape(-1) == pad, idx[q], inv[q], cnt[q], off[q], B, L)


def test_combine_rows():
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(5)
    M, d = 3001, 256
    ma, mb = torch.rand(M, generator=g) < 0.4, torch.rand(M, generator=g) < 0.6
    inv_a = torch.full((M,), -1, dtype=torch.int32)
    inv_a[ma] = torch.arange(int(ma.sum()), dtype=torch.int32)
    inv_b = torch.full((M,), -1, dtype=torch.int32)
    inv_b[mb] = torch.arange(int(mb.sum()), dtype=torch.int32)
    a, b = torch.randn(int(ma.sum()), d, generator=g), torch.randn(int(mb.sum()), d, generator=g)
    out = torch.empty(M, d, device=DEV)
    lib('c2dsr_combine_rows', a.to(DEV), inv_a.to(DEV), b.to(DEV), inv_b.to(DEV), M, d, out, stream())
    want = torch.zeros(M, d)
    want[ma] += a
    want[mb] += b
    assert torch.equal(out.cpu(), want)


@pytest.mark.parametrize('M', [1, 1000, 1024, 40960])
def test_compact_valid_targets(M):
    from c2dsr_amd._lib import lib, stream
    g = np.random.default_rng(M)
    ignore = 99
    t = g.integers(0, 100, M)
    t[g.random(M) < 0.4] = ignore
    split = M // 2
    tt = torch.from_numpy(t).to(DEV)
    idx = torch.empty(M, device=DEV, dtype=torch.int32)
    inv = torch.empty(M, device=DEV, dtype=torch.int32)
    tc = torch.empty(M, device=DEV, dtype=torch.int64)
    cnt = torch.empty(2, device=DEV, dtype=torch.int32)
    ws = torch.empty(lib.raw('c2dsr_compact_workspace')(M, 1) // 4 + 1, device=DEV, dtype=torch.int32)
    lib('c2dsr_compact_valid', tt, M, split, ignore, idx, inv, tc, cnt, ws, None, stream())
    want = np.nonzero(t != ignore)[0]
    n = len(want)
    assert cnt.tolist() == [int((want < split).sum()), int((want >= split).sum())]
    assert np.array_equal(idx[:n].cpu().numpy(), want)
    assert np.array_equal(tc[:n].cpu().numpy(), t[want])
    winv = np.full(M, -1)
    winv[want] = np.arange(n)
    assert np.array_equal(inv.cpu().numpy(), winv)


# ----------------------------------------------------------------------------- bf16 dqkv hand-off
@pytest.mark.parametrize('B,L,d,H,p', [(13, 50, 256, 1, 0.2), (6, 64, 64, 2, 0.0), (4, 8, 32, 1, 0.1)])
def test_attention_bwd_b16_is_the_rounded_fp32_dqkv(B, L, d, H, p):
    """c2dsr_attn_bwd_b16 writes exactly bf16(RNE) of what c2dsr_attn_bwd writes in fp32."""
    from c2dsr_amd._lib import lib, stream
    torch.manual_seed(B + L + d)
    pad = 999
    seq = torch.randint(0, 900, (B, L))
    for b in range(B):
        seq[b, :L - int(torch.randint(1, L, (1,)))] = pad
    seq[:, 0] = pad
    sd = seq.to(DEV)
    qkv = torch.randn(B, L, 3 * d, device=DEV)
    dout = torch.randn(B, L, d, device=DEV)
    P = torch.empty(int(lib.raw('c2dsr_attn_psave_floats')(B, L, d, H)), device=DEV)
    out = torch.empty(B, L, d, device=DEV)
    s = stream()
    assert bool(lib.raw('c2dsr_attn_bwd_b16_supported')(L, d, H))
    lib('c2dsr_attn_fwd', qkv, sd, pad, B, L, d, H, 11, 22, p, 3, out, P, s)
    g32 = torch.empty_like(qkv)
    lib('c2dsr_attn_bwd', qkv, sd, pad, B, L, d, H, 11, 22, p, 3, P, dout, g32, s)
    g16 = torch.empty(qkv.shape, device=DEV, dtype=torch.bfloat16)
    lib('c2dsr_attn_bwd_b16', qkv, sd, pad, B, L, d, H, 11, 22, p, 3, P, dout, g16, s)
    torch.cuda.synchronize()
    assert torch.equal(g16, g32.to(torch.bfloat16))


@pytest.mark.parametrize('aux', [0, 1, 3])
def test_rgemm_b16a_equals_fp32_path(aux):
    """The in_proj dX over a bf16 dqkv equals the fp32-A call on the same (bf16-valued) operand, bit for bit,
    in every aux mode the backward uses (none, in-place residual sum, mapped row-subset sum)."""
    from c2dsr_amd.ops import AUX_ACC, AUX_ACC_MAP, rgemm, to_bf16
    M, N, K = 1037, 256, 768
    g = torch.Generator().manual_seed(aux)
    A16 = torch.randn(M, K, generator=g).to(DEV).to(torch.bfloat16)
    Wb = to_bf16(torch.randn(K, N, generator=g).to(DEV), trans=True)
    kw = {}
    if aux == 1:
        base = torch.randn(M, N, generator=g).to(DEV)
    elif aux == 3:
        n_sub = 300
        auxmap = torch.full((M,), -1, dtype=torch.int32)
        auxmap[torch.randperm(M, generator=g)[:n_sub]] = torch.arange(n_sub, dtype=torch.int32)
        park = torch.randn(n_sub, N, generator=g).to(DEV)
        kw = dict(aux_mode=AUX_ACC_MAP, aux=park, auxmap=auxmap.to(DEV))
    outs = []
    for A in (A16, A16.float()):
        if aux == 1:
            C = base.clone()
            rgemm(A, Wb, C, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C)
        else:
            C = torch.empty(M, N, device=DEV)
            rgemm(A, Wb, C, M=M, N=N, K=K, **kw)
        outs.append(C)
    torch.cuda.synchronize()
    dif = (outs[0] - outs[1]).abs()
    bad = torch.nonzero(dif > 0)
    assert torch.equal(outs[0], outs[1]), (f'{bad.shape[0]} differ, max {float(dif.max())}, rows '
                                           f'{bad[:, 0].unique()[:20].tolist()}, cols {bad[:, 1].unique()[:20].tolist()}, '
                                           f'ref scale {float(outs[1].abs().max())}')


def test_wgemm_b16y_equals_fp32_path():
    from c2dsr_amd.ops import wgemm
    T, N, D = 4097, 768, 256
    g = torch.Generator().manual_seed(7)
    dY16 = torch.randn(T, N, generator=g).to(DEV).to(torch.bfloat16)
    X = torch.randn(T, D, generator=g).to(DEV)
    res = []
    for dY in (dY16, dY16.float()):
        dW = torch.full((N, D), 0.5, device=DEV)
        db = torch.full((N,), 0.25, device=DEV)
        wgemm(dY, X, dW, T=T, N=N, D=D, beta=1.0, db=db)
        res.append((dW, db))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_gemm_split_k_deterministic():
    """Split-K (the bilinear weight gradient: M = N = d, K = B) sums its partial slabs in split order: the
    same bits on every run, no float atomics."""
    from c2dsr_amd.ops import gemm
    M, N, K = 256, 256, 4096
    g = torch.Generator().manual_seed(3)
    A, B, C0 = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g), torch.randn(M, N, generator=g)
    outs = []
    for _ in range(3):
        C = C0.to(DEV)
        gemm(A.to(DEV), B.to(DEV), C, M=M, N=N, K=K, transA=1, beta=1.0, split_k=0)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert rel(outs[0], C0.double() + A.double().T @ B.double()) < 1e-5


# ----------------------------------------------------------------------------- row-subset attention
def _rows_case(B, L, seed, q_frac):
    """Sequences with padding anywhere (left-padded, scattered, none, all) and a query-row subset."""
    g = np.random.default_rng(seed)
    pad = 999
    seq = g.integers(0, 900, (B, L))
    for b in range(B):
        kind = b % 4
        if kind == 0:
            seq[b, :g.integers(0, L + 1)] = pad
        elif kind == 1:
            seq[b, g.random(L) < 0.5] = pad
        elif kind == 2 and b % 8 == 2:
            seq[b, :] = pad
        # kind 3 / the rest: no padding
    need = g.random((B, L)) < q_frac
    need[:, -3:] = True
    need[B // 2] = False  # a sequence with no query row
    return pad, seq, need


def _row_set(mask):
    from c2dsr_amd.ops import RowSet
    B, L = mask.shape
    flat = mask.reshape(-1)
    idx = np.nonzero(flat)[0].astype(np.int32)
    inv = np.full(B * L, -1, np.int32)
    inv[idx] = np.arange(len(idx), dtype=np.int32)
    off = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
    t = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    return RowSet(t(idx), t(inv), len(idx), B * L, t(off)), idx


@pytest.mark.parametrize('B,L,d,H,p,q_frac', [(64, 50, 256, 1, 0.2, 0.4), (40, 64, 256, 2, 0.0, 0.9),
                                              (24, 32, 64, 2, 0.3, 0.5), (9, 64, 32, 1, 0.1, 0.2)])
def test_attention_rows_equals_full_layout(B, L, d, H, p, q_frac):
    """c2dsr_attn_fwd_rows / _bwd_rows (queries = a row subset, keys = the padding rows, compact) against the
    full-layout wave kernels on the same q / k / v: the output and dq at the query rows, dk / dv at the
    padding rows (the full layout's other rows of dk / dv are 0 when dout is 0 off the query rows)."""
    from c2dsr_amd._lib import lib, stream
    pad, seq, need = _rows_case(B, L, B * L + d, q_frac)
    rs, qi = _row_set(need)
    ks, ki = _row_set(seq == pad)
    torch.manual_seed(B)
    qkv = torch.randn(B * L, 3 * d, device=DEV)
    dout_c = torch.randn(len(qi), d, device=DEV)
    dout = torch.zeros(B * L, d, device=DEV)
    dout[torch.from_numpy(qi).long().to(DEV)] = dout_c
    sd = torch.from_numpy(seq).to(DEV)
    s = stream()
    nP = int(lib.raw('c2dsr_attn_psave_floats')(B, L, d, H))
    P, Pr = torch.empty(nP, device=DEV), torch.empty(nP, device=DEV)
    out = torch.empty(B * L, d, device=DEV)
    lib('c2dsr_attn_fwd', qkv, sd, pad, B, L, d, H, 5, 6, p, 2, out, P, s)
    g = torch.empty_like(qkv)
    lib('c2dsr_attn_bwd', qkv, sd, pad, B, L, d, H, 5, 6, p, 2, P, dout, g, s)
    qL, kL = torch.from_numpy(qi).long().to(DEV), torch.from_numpy(ki).long().to(DEV)
    # compact q / kv whose storage ENDS at the last row (a read past the last sequence's rows would leave the
    # allocation: the round-1 attention fault's shape, for the row-subset kernels)
    q = _tail_of_segment(qkv[qL, :d].contiguous().cpu())
    kv = _tail_of_segment(qkv[kL, d:].contiguous().cpu())
    out_r = torch.empty(len(qi), d, device=DEV)
    lib('c2dsr_attn_fwd_rows', q, kv, sd, pad, rs.idx, rs.off, ks.idx, ks.off, B, L, d, H, 5, 6, p, 2, out_r, Pr, s)
    dq = torch.full((len(qi), d), 7.0, device=DEV)
    dkv = torch.full((len(ki), 2 * d), 7.0, device=DEV)
    lib('c2dsr_attn_bwd_rows', q, kv, sd, pad, rs.idx, rs.off, ks.idx, ks.off, B, L, d, H, 5, 6, p, 2, Pr, dout_c,
        dq, dkv, 0, s)
    dq16 = torch.empty(len(qi), d, device=DEV, dtype=torch.bfloat16)
    dkv16 = torch.empty(len(ki), 2 * d, device=DEV, dtype=torch.bfloat16)
    lib('c2dsr_attn_bwd_rows', q, kv, sd, pad, rs.idx, rs.off, ks.idx, ks.off, B, L, d, H, 5, 6, p, 2, Pr, dout_c,
        dq16, dkv16, 1, s)
    torch.cuda.synchronize()
    assert rel(out_r, out[qL]) < 2e-6
    assert rel(dq, g[qL, :d]) < 2e-6
    assert rel(dkv, g[kL, d:]) < 2e-6
    assert torch.equal(dq16, dq.to(torch.bfloat16)) and torch.equal(dkv16, dkv.to(torch.bfloat16))
    # rows with no admissible key (no padding at or before them) are exactly 0 in both
    assert torch.equal(out_r[out[qL].abs().amax(1) == 0], torch.zeros_like(out_r[out[qL].abs().amax(1) == 0]))


@pytest.mark.parametrize('K,aux', [(256, 0), (256, 1), (512, 0)])
def test_rgemm_b16a_row_subset_shapes(K, aux):
    """bf16-A dX products of the row-subset layer (dq: K = 256 with the parked LN gradient, dkv: K = 512) equal
    the fp32-A call bit for bit."""
    from c2dsr_amd.ops import AUX_ACC, rgemm, to_bf16
    M, N = 2113, 256
    g = torch.Generator().manual_seed(K + aux)
    A16 = torch.randn(M, K, generator=g).to(DEV).to(torch.bfloat16)
    Wb = to_bf16(torch.randn(K, N, generator=g).to(DEV), trans=True)
    base = torch.randn(M, N, generator=g).to(DEV)
    outs = []
    for A in (A16, A16.float()):
        C = base.clone()
        if aux:
            rgemm(A, Wb, C, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C)
        else:
            rgemm(A, Wb, C, M=M, N=N, K=K)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_to_bf16_multi_equals_single():
    """The batched weight-image conversion (one launch per optimizer step) writes exactly what c2dsr_to_bf16
    writes per matrix (plain and transposed, a strided source, an empty matrix)."""
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import to_bf16
    g = torch.Generator().manual_seed(1)
    big = torch.randn(300, 520, generator=g).to(DEV)
    mats = [(torch.randn(256, 256, generator=g).to(DEV), 0), (torch.randn(512, 256, generator=g).to(DEV), 1),
            (big[:, :300], 1), (big[10:, 8:], 0), (torch.empty(0, 256, device=DEV), 0), (torch.randn(3, 5, generator=g).to(DEV), 1)]
    outs, recs = [], []
    for X, tr in mats:
        R, C = X.shape
        y = torch.empty((C, R) if tr else (R, C), device=DEV, dtype=torch.bfloat16)
        outs.append(y)
        recs += [X.data_ptr(), y.data_ptr(), R, C, X.stride(0), tr]
    desc = np.asarray(recs, dtype=np.int64)
    lib('c2dsr_to_bf16_multi', desc, len(mats), stream())
    torch.cuda.synchronize()
    for (X, tr), y in zip(mats, outs):
        if X.numel():
            assert torch.equal(y, to_bf16(X, bool(tr)))


@pytest.mark.parametrize('M,N,strided', [(40960, 256, True), (1000, 37, False), (3, 256, True)])
def test_weighted_colsum(M, N, strided):
    """c2dsr_wcolsum (the classifier_pad weight gradient: Σ_r w_r·H[r, :], w a strided column) and plain
    c2dsr_colsum against float64, and bitwise reproducible."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(M + N)
    X = torch.randn(M, N, generator=g)
    wfull = torch.randn(M, 5, generator=g)
    w, ldw = (wfull[:, 3], 5) if strided else (wfull[:, 0].contiguous(), 1)
    out0 = torch.randn(N, generator=g)
    ws = torch.empty(lib.raw('c2dsr_colsum_workspace')(M, N), dtype=torch.uint8, device=DEV)
    Xd, wd = X.to(DEV), wfull.to(DEV)
    wptr = wd[:, 3] if strided else wd[:, 0].contiguous()
    res = []
    for _ in range(2):
        out = out0.to(DEV)
        lib('c2dsr_wcolsum', Xd, M, N, N, wptr, ldw, 0.5, 1.0, out, ws, stream())
        res.append(out)
    plain = out0.to(DEV)
    lib('c2dsr_colsum', Xd, M, N, N, 1.0, 0.0, plain, ws, stream())
    torch.cuda.synchronize()
    ref = out0.double() + 0.5 * (w.double()[:, None] * X.double()).sum(0)
    assert rel(res[0], ref) < 1e-5 and torch.equal(res[0], res[1])
    assert rel(plain, X.double().sum(0)) < 1e-5


@pytest.mark.parametrize('n,nparts', [(16 * 1024 * 256, 3), (1001, 2), (64000, 1)])
def test_sum_parts(n, nparts):
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(n)
    part = torch.randn(nparts, n, generator=g)
    out0 = torch.randn(n, generator=g)
    out = out0.to(DEV)
    lib('c2dsr_sum_parts', part.to(DEV), nparts, n, 1.0, out, stream())
    t = torch.zeros(n)
    for s_ in range(nparts):  # the kernel's order: the parts summed in split order, then added to beta·out
        t += part[s_]
    assert torch.equal(out.cpu(), out0 + t)


@pytest.mark.parametrize('rows,d,p,mapped', [(3001, 256, 0.2, True), (517, 64, 0.0, False), (64, 512, 0.1, False)])
def test_add_ln2_equals_two_layernorms(rows, d, p, mapped):
    """c2dsr_add_ln2_fwd / _ln2_bwd (norm2 + the encoder's final norm in one pass) against the two
    c2dsr_add_ln_fwd / c2dsr_ln_bwd calls they replace: outputs, input gradients and all four parameter
    gradients."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(rows + d)
    t = lambda *sh: torch.randn(*sh, generator=g).to(DEV)  # noqa: E731
    a, b, dy = t(rows, d), t(rows, d), t(rows, d)
    w2, b2, wF, bF = t(d) * 0.5 + 1, t(d) * 0.1, t(d) * 0.5 + 1, t(d) * 0.1
    keys, base = (7, 9), 11
    rowmap = torch.sort(torch.randperm(4 * rows, generator=g)[:rows])[0].to(torch.int32).to(DEV) if mapped else None
    s = stream()
    f32 = dict(device=DEV, dtype=torch.float32)
    # reference: two calls
    xs, x2, m2, r2 = (torch.empty(rows, d, **f32), torch.empty(rows, d, **f32), torch.empty(rows, **f32),
                      torch.empty(rows, **f32))
    lib('c2dsr_add_ln_fwd', a, b, rows, d, keys[0], keys[1], p, base, rowmap, w2, b2, 1e-8, xs, x2, m2, r2, s)
    y, mF, rF = torch.empty(rows, d, **f32), torch.empty(rows, **f32), torch.empty(rows, **f32)
    lib('c2dsr_add_ln_fwd', x2, None, rows, d, 0, 0, 0.0, 0, None, wF, bF, 1e-8, None, y, mF, rF, s)
    ws = torch.empty(lib.raw('c2dsr_ln_bwd_workspace')(d), dtype=torch.uint8, device=DEV)
    gr = [torch.zeros(d, **f32) for _ in range(4)]
    dx2 = torch.empty(rows, d, **f32)
    lib('c2dsr_ln_bwd', x2, mF, rF, wF, dy, rows, d, dx2, 0, None, 0, 0, 0.0, 0, None, gr[2], gr[3], ws, s)
    da, db = torch.empty(rows, d, **f32), torch.empty(rows, d, **f32)
    lib('c2dsr_ln_bwd', xs, m2, r2, w2, dx2, rows, d, da, 0, db, keys[0], keys[1], p, base, rowmap, gr[0], gr[1], ws,
        s)
    # fused
    xs2, y2, st = torch.empty(rows, d, **f32), torch.empty(rows, d, **f32), torch.empty(4, rows, **f32)
    lib('c2dsr_add_ln2_fwd', a, b, rows, d, keys[0], keys[1], p, base, rowmap, w2, b2, 1e-8, wF, bF, 1e-8, xs2, y2,
        st, s)
    ws2 = torch.empty(lib.raw('c2dsr_ln2_bwd_workspace')(d), dtype=torch.uint8, device=DEV)
    gf = [torch.zeros(d, **f32) for _ in range(4)]
    da2, db2 = torch.empty(rows, d, **f32), torch.empty(rows, d, **f32)
    lib('c2dsr_ln2_bwd', xs2, st, w2, b2, wF, dy, rows, d, da2, db2, keys[0], keys[1], p, base, rowmap, *gf, ws2, s)
    torch.cuda.synchronize()
    assert torch.equal(xs2, xs)
    for u, v in [(y2, y), (da2, da), (db2, db)] + list(zip(gf, gr)):
        assert rel(u, v) < 1e-6


@pytest.mark.parametrize('b16', [False, True])
def test_wgemm_multi_segments(b16):
    """c2dsr_wgemm_multi (one weight-gradient product over the row sets of several passes, ops.WGradBatch)
    against float64 Σ_k dY_kᵀ·X_k of the bf16-rounded operands, segments of ragged lengths (not multiples of
    32), with the bias column sums; deterministic."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(11 + b16)
    N, D = 512, 256
    Ts = (1000, 33, 4097)
    dYs = [torch.randn(T, N, generator=g) for T in Ts]
    Xs = [torch.randn(T, D, generator=g) for T in Ts]
    dYd = [y.to(DEV).to(torch.bfloat16) if b16 else y.to(DEV) for y in dYs]
    Xd = [x.to(DEV) for x in Xs]
    ws = torch.empty(lib.raw('c2dsr_wgemm_workspace')(N), dtype=torch.uint8, device=DEV)
    desc = np.asarray([v for y, x, T in zip(dYd, Xd, Ts) for v in (y.data_ptr(), N, x.data_ptr(), D, T)],
                      dtype=np.int64)
    outs = []
    for _ in range(2):
        dW = torch.full((N, D), 0.5, device=DEV)
        db = torch.full((N,), 0.25, device=DEV)
        lib('c2dsr_wgemm_multi', desc, len(Ts), N, D, int(b16), 1.0, dW, db, ws, stream())
        outs.append((dW, db))
    torch.cuda.synchronize()
    r = lambda t: t.to(torch.bfloat16).double()  # noqa: E731  (the MFMA operands)
    refW = 0.5 + sum(r(y).T @ r(x) for y, x in zip(dYs, Xs))
    refb = 0.25 + sum((r(y) if b16 else y.double()).sum(0) for y in dYs)
    assert rel(outs[0][0], refW) < 2e-3 and rel(outs[0][1], refb) < 1e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_bilinear_ds_equals_rowscale_products():
    """c2dsr_bilinear_ds (both discriminators' row-scale products of the MI-loss backward in one launch) equals the
    separately rounded products and their sum, bit for bit (torch elementwise ops as the reference)."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(5)
    B, d = 1000, 256
    Ua, Ub = torch.randn(2 * B, d, generator=g), torch.randn(2 * B, d, generator=g)
    xa, xb = torch.randn(B, d, generator=g), torch.randn(B, d, generator=g)
    dS = torch.randn(4, B, generator=g)
    dev = [t.to(DEV) for t in (Ua, Ub, xa, xb, dS)]
    out = [torch.empty(B, d, device=DEV), torch.empty(B, d, device=DEV), torch.empty(2 * B, d, device=DEV),
           torch.empty(2 * B, d, device=DEV)]
    lib('c2dsr_bilinear_ds', *dev, B, d, *out, stream())
    torch.cuda.synchronize()
    for j, (U, x) in enumerate(((Ua, xa), (Ub, xb))):
        s0, s1 = dS[2 * j][:, None], dS[2 * j + 1][:, None]
        assert torch.equal(out[j].cpu(), (s0 * U[:B]) + (s1 * U[B:]))
        assert torch.equal(out[2 + j].cpu(), torch.cat([s0 * x, s1 * x]))


def test_mi_scores_equals_four_rowdots():
    """c2dsr_mi_scores (the four discriminator scores in one launch) equals four c2dsr_rowdot calls bit for bit."""
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(6)
    B, d = 777, 256
    x1a, x1b = torch.randn(B, d, generator=g).to(DEV), torch.randn(B, d, generator=g).to(DEV)
    Ua, Ub = torch.randn(2 * B, d, generator=g).to(DEV), torch.randn(2 * B, d, generator=g).to(DEV)
    ba, bb = torch.randn(1, generator=g).to(DEV), None
    S = torch.empty(4, B, device=DEV)
    lib('c2dsr_mi_scores', x1a, Ua, ba, x1b, Ub, bb, B, d, S, stream())
    R = torch.empty(4, B, device=DEV)
    lib('c2dsr_rowdot', x1a, d, Ua, d, B, d, ba, R[0], 1, stream())
    lib('c2dsr_rowdot', x1a, d, Ua[B:], d, B, d, ba, R[1], 1, stream())
    lib('c2dsr_rowdot', x1b, d, Ub, d, B, d, bb, R[2], 1, stream())
    lib('c2dsr_rowdot', x1b, d, Ub[B:], d, B, d, bb, R[3], 1, stream())
    torch.cuda.synchronize()
    assert torch.equal(S, R)
