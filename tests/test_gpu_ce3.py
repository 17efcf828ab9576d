"""K5 at reference precision (csrc/ce3.hip): the fused classifier head + cross-entropy on split-bf16
operands (hi + lo, three bf16 MFMAs per product, fp32 accumulation) against a float64 computation of the
same op on the SAME fp32 operands (no rounding of the inputs): the fp32 training mode's tolerance.

Reference semantics: trainer.py:131-154 (logits = h·Wᵀ + b ‖ pad column, cross_entropy with
ignore_index = n) — forward lse / per-row loss, dH = rw·(softmax − onehot)·W, dW = Σ_r rw·(softmax −
onehot)ᵀ·H, db likewise."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _run(H, W, b, pl, t, coef, lam, ns, nr, BR, g0=None, b16=False, lgk=False):
    """The head exactly as losshead.py drives it: the fp32 mode's x3 kernels (split-bf16 images), or with
    b16 the bf16 mode's ce3b kernels (plain bf16 images, zero rows to whole 64-row tiles); lgk: the fp32 mode with
    the logits stored by the forward and the dW sweeps reading them (c2dsr_ce3_fused_fwd_u_lg / _dw_lg*)."""
    from c2dsr_amd._lib import lib, stream
    s = stream()
    d = lambda x: x.to(DEV)  # noqa: E731
    M, D = H.shape
    n = W.shape[0]
    M_pad = max(64, -(-M // 64) * 64)
    pre = 'c2dsr_ce3b_fused_' if b16 else 'c2dsr_ce3_fused_'
    if b16:
        n64 = -(-n // 64) * 64
        Hx = torch.zeros(M_pad, D, dtype=torch.bfloat16, device=DEV)
        Wx = torch.zeros(n64, D, dtype=torch.bfloat16, device=DEV)
        lib('c2dsr_f32_to_bf16', d(H), M * D, Hx, s)
        lib('c2dsr_f32_to_bf16', d(W), n * D, Wx, s)
    else:
        n32 = -(-n // 32) * 32
        Hx = torch.empty(M_pad, 2 * D, dtype=torch.bfloat16, device=DEV)
        Wx = torch.empty(n32, 2 * D, dtype=torch.bfloat16, device=DEV)
        lib('c2dsr_f32_split_bf16', d(H), M, D, M_pad, Hx, s)
        lib('c2dsr_f32_split_bf16', d(W), n, D, n32, Wx, s)
    n_pad = -(-n // 128) * 128 + 64
    bias2 = torch.empty(n_pad, device=DEV)
    lib('c2dsr_ce_bias2', d(b), n, n_pad, bias2, s)
    pm, ps = torch.empty(ns, M, device=DEV), torch.empty(ns, M, device=DEV)
    Up = torch.empty(ns, M, D, device=DEV)
    lse, rows = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    lse2 = torch.empty(M_pad, device=DEV)
    if lgk:
        lg = torch.full((int(lib.raw('c2dsr_ce3_logits_floats')(M, n)),), float('nan'), device=DEV)
        lib(pre + 'fwd_u_lg', Hx, Wx, bias2, M, n, D, ns, pm, ps, Up, d(pl), d(t), d(H), d(W), d(b), lse, lse2,
            rows, lg, s)
        # the dW sweeps on the stored logits, same call shapes as the recomputing ones
        dw = lambda Hx_, Wx_, b2_, M_, n_, D_, nr_, crow_, o1, o2, s_, col0=0: lib(  # noqa: E731
            pre + 'dw_lg', Hx_, lg, M_, n, col0, n_, D_, nr_, crow_, o1, o2, s_)
    else:
        lib(pre + 'fwd_u', Hx, Wx, bias2, M, n, D, ns, pm, ps, Up, d(pl), d(t), d(H), d(W), d(b), lse, lse2,
            rows, s)
        dw = lambda *a, col0=0: lib(pre + 'dw', *a)  # noqa: E731
    rw, dpad = torch.empty(M_pad, device=DEV), torch.empty(M, device=DEV)
    t32 = torch.empty(M_pad, device=DEV, dtype=torch.int32)
    crow = torch.empty(M_pad + 64, device=DEV)
    gs = torch.tensor([1.0])
    lib('c2dsr_ce_row_weights', d(t), M, M_pad, n, d(coef), BR, d(gs), lam, d(pl), lse, rw, t32, lse2, crow, dpad, s)
    dH = torch.empty(M, D, device=DEV)
    lib('c2dsr_ce_dh_from_u', Up, pm, ns, M, D, lse2, t32, rw, d(W), n, dH, s)
    gW = torch.zeros(n, D, device=DEV) if g0 is None else g0[0].clone().to(DEV)
    gb = torch.zeros(n, device=DEV) if g0 is None else g0[1].clone().to(DEV)
    if nr <= -2:  # whole rounds of row blocks added directly, the remainder's row blocks split -nr ways and summed
        from c2dsr_amd.losshead import dw_full_rows
        full = dw_full_rows(n, not b16)  # whole rounds of the instantiation's row blocks (128 / 192 rows)
        rem, k = n - full, -nr
        ic = Wx.shape[1]
        dw(Hx, Wx, bias2, M, full, D, 0, crow, gW, gb, s)
        dWp, dbp = torch.empty(k, rem, D, device=DEV), torch.empty(k, rem, device=DEV)
        dw(Hx, Wx.view(-1)[full * ic:], bias2[full:], M, rem, D, k, crow, dWp, dbp, s, col0=full)
        lib('c2dsr_sum_parts', dWp, k, rem * D, 1.0, gW.view(-1)[full * D:], s)
        lib('c2dsr_sum_parts', dbp, k, rem, 1.0, gb[full:], s)
    elif nr == -1:  # stream-K sweep (whole row blocks added directly, split ones combined in workgroup order)
        wsb = int(lib.raw('c2dsr_ce3_dw_sk_workspace')(D))
        ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
        if lgk:
            lib(pre + 'dw_lg_sk', Hx, lg, M, n, D, crow, gW, gb, ws, wsb, s)
        else:
            lib(pre + 'dw_sk', Hx, Wx, bias2, M, n, D, crow, gW, gb, ws, wsb, s)
    elif nr == 0:  # one split added straight onto the gradients
        dw(Hx, Wx, bias2, M, n, D, 0, crow, gW, gb, s)
    else:
        dWp, dbp = torch.empty(nr, n, D, device=DEV), torch.empty(nr, n, device=DEV)
        dw(Hx, Wx, bias2, M, n, D, nr, crow, dWp, dbp, s)
        lib('c2dsr_sum_parts', dWp, nr, n * D, 1.0, gW, s)
        lib('c2dsr_sum_parts', dbp, nr, n, 1.0, gb, s)
    wsb = int(lib.raw('c2dsr_ce_onehot_workspace')(M, n, D))
    ws = torch.empty(wsb, device=DEV, dtype=torch.uint8)
    lib('c2dsr_ce_onehot_dw', d(t), M, n, d(H), D, rw, gW, gb, ws, wsb, s)
    torch.cuda.synchronize()
    return lse, rows, dH, gW, gb, dpad, Up


def _ref(H, W, b, pl, t, coef, lam, BR):
    M = H.shape[0]
    n = W.shape[0]
    lg = torch.cat([H.double() @ W.double().T + b.double(), pl.double()[:, None]], 1)
    lse = torch.logsumexp(lg, 1)
    valid = t != n
    rows = torch.where(valid, lse - lg.gather(1, t[:, None])[:, 0], torch.zeros(M, dtype=torch.float64))
    w_r = torch.where(valid, lam * coef[(torch.arange(M) >= BR).long()].double(), torch.zeros(M, dtype=torch.float64))
    P = torch.softmax(lg, 1)
    oh = torch.zeros_like(P)
    oh[torch.arange(M), t] = 1.0
    dl = (P - oh) * w_r[:, None]
    return lse, rows, dl[:, :n] @ W.double(), dl[:, :n].T @ H.double(), dl[:, :n].sum(0), dl[:, n]


# fp32-mode tolerances: split-bf16 products carry ≈3·2^-17 relative error per term (see ce3.hip), so a
# logit over d = 256 terms is off by ~1e-5 of Σ|h·w| (fp32: ~1e-6); north_star's bound is 1e-4 relative.
# lse within 1e-5 relative, per-row losses and every gradient within 5e-5 of their max-abs.
TOL_LSE, TOL = 1e-5, 5e-5


@pytest.mark.parametrize('M,n,D,ns,nr', [(300, 700, 256, 3, 2), (1000, 2100, 128, 4, 3), (64, 65, 256, 1, 1),
                                         (777, 4099, 256, 7, 5), (33, 31, 256, 2, 3), (300, 700, 256, 3, -1),
                                         (1000, 2100, 128, 4, -1), (2500, 40000, 256, 5, -1), (33, 31, 256, 2, -1),
                                         (700, 36845, 256, 3, -8)])
@pytest.mark.parametrize('lgk', [False, True])
def test_ce3_matches_float64(M, n, D, ns, nr, lgk):
    g = torch.Generator().manual_seed(M + n + D)
    H = torch.randn(M, D, generator=g) * 0.5
    W = torch.randn(n, D, generator=g) * 0.5
    b = torch.randn(n, generator=g) * 0.1
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n + 1, (M,), generator=g)
    t[:5] = n  # ignored rows
    coef, lam, BR = torch.tensor([0.37, 1.9]), 0.7, M // 2
    lse, rows, dH, gW, gb, dpad, _ = _run(H, W, b, pl, t, coef, lam, ns, nr, BR, lgk=lgk)
    lse_r, rows_r, dH_r, gW_r, gb_r, dpad_r = _ref(H, W, b, pl, t, coef, lam, BR)
    err = dict(lse=rel(lse, lse_r), rows=rel(rows, rows_r), dpad=rel(dpad, dpad_r), dH=rel(dH, dH_r),
               gW=rel(gW, gW_r), gb=rel(gb, gb_r))
    print('ce3 errors', {k: f'{v:.2e}' for k, v in err.items()})
    assert err.pop('lse') < TOL_LSE
    assert all(v < TOL for v in err.values()), err


@pytest.mark.parametrize('M,n,D,ns', [(200, 1500, 256, 2), (333, 3000, 128, 5)])
@pytest.mark.parametrize('lgk', [False, True])
def test_ce3_online_rescale(M, n, D, ns, lgk):
    """Row max rising and falling across column tiles (bias ramp of 60 nats): the lazy rescale fires at
    different tiles for different rows of one wave.  The logits reach |h·w| ≈ 20 here, and the softmax's
    relative error is the logit's ABSOLUTE error (≈ 4e-6·|h·w| for split-bf16 products), so the weight
    gradient is held to north_star's 1e-4 instead of TOL."""
    g = torch.Generator().manual_seed(M * 7 + n)
    H = torch.randn(M, D, generator=g) * 0.3
    H[1::2, :8] = -H[1::2, :8].abs() - 1.0
    H[0::2, :8] = H[0::2, :8].abs() + 1.0
    W = torch.randn(n, D, generator=g) * 0.2
    W[:, :8] = torch.linspace(-2.0, 2.0, n)[:, None]
    b = torch.linspace(0.0, 60.0, n) * (torch.rand(n, generator=g) > 0.5)
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n, (M,), generator=g)
    coef, lam, BR = torch.tensor([0.5, 1.5]), 0.7, M // 2
    lse, rows, dH, gW, gb, _, Up = _run(H, W, b, pl, t, coef, lam, ns, 2, BR, lgk=lgk)
    lse_r, rows_r, dH_r, gW_r, gb_r, _ = _ref(H, W, b, pl, t, coef, lam, BR)
    assert torch.isfinite(Up).all()
    err = dict(lse=rel(lse, lse_r), rows=rel(rows, rows_r), dH=rel(dH, dH_r), gW=rel(gW, gW_r), gb=rel(gb, gb_r))
    print('ce3 rescale errors', {k: f'{v:.2e}' for k, v in err.items()})
    assert err.pop('lse') < TOL_LSE
    assert all(v < 1e-4 for v in err.values()), err


@pytest.mark.parametrize('lgk', [False, True])
def test_ce3_dw_accumulates_onto_gradient(lgk):
    """n_rsplit = 0 (one split, losshead.py when split_count(n) == 1): the dW / db sweep adds onto the existing
    gradient buffers (the epoch-long accumulation, Q3) and equals the partial + sum path bit for bit."""
    M, n, D = 500, 2100, 256
    g = torch.Generator().manual_seed(99)
    H = torch.randn(M, D, generator=g) * 0.5
    W = torch.randn(n, D, generator=g) * 0.5
    b = torch.randn(n, generator=g) * 0.1
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n + 1, (M,), generator=g)
    coef = torch.tensor([0.37, 1.9])
    g0 = (torch.randn(n, D, generator=g), torch.randn(n, generator=g))
    r1 = _run(H, W, b, pl, t, coef, 0.7, 3, 0, M // 2, g0=g0, lgk=lgk)
    r2 = _run(H, W, b, pl, t, coef, 0.7, 3, 1, M // 2, g0=g0, lgk=lgk)
    assert torch.equal(r1[3], r2[3]) and torch.equal(r1[4], r2[4])
    assert not torch.equal(r1[3].cpu(), g0[0])


def test_split_bf16_is_exact_to_2e17():
    from c2dsr_amd._lib import lib, stream
    g = torch.Generator().manual_seed(5)
    x = torch.randn(70, 256, generator=g) * torch.logspace(-3, 3, 256)
    out = torch.full((96, 512), 7.0, dtype=torch.bfloat16, device=DEV)
    lib('c2dsr_f32_split_bf16', x.to(DEV), 70, 256, 96, out, stream())
    torch.cuda.synchronize()
    o = out.float().cpu()
    hi, lo = o[:70, :256], o[:70, 256:]
    assert torch.equal(hi, x.to(torch.bfloat16).float())
    assert float(((hi.double() + lo.double() - x.double()).abs() / x.double().abs()).max()) <= 2 ** -17
    assert torch.equal(o[70:], torch.zeros(26, 512))


# ---------------------------------------------------------------- fp32-mode projections (csrc/rgemm.hip, X3)
@pytest.mark.parametrize('M,N,K', [(1000, 768, 256), (129, 256, 256), (77, 320, 512), (32 * 37 + 5, 256, 512)])
def test_rgemm_x3_matches_float64(M, N, K):
    """Split-bf16 row-streaming GEMM on unrounded fp32 operands vs float64: plain, bias + alpha, and every aux
    epilogue (in-place accumulate, drop(relu)-backward mask, mapped accumulate) at the fp32-mode tolerance."""
    from c2dsr_amd.ops import AUX_ACC, AUX_ACC_MAP, AUX_MASK, rgemm, to_split_bf16
    g = torch.Generator().manual_seed(M + N + K)
    A, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    Wx = to_split_bf16(W.to(DEV))
    prod = A.double() @ W.double().T
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), Wx, C, M=M, N=N, K=K, alpha=0.5, bias=b.to(DEV), x3=True)
    assert rel(C, 0.5 * prod + b.double()) < TOL
    Wt = torch.randn(K, N, generator=g)  # transposed image (the dx = dy·W product)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), to_split_bf16(Wt.to(DEV), trans=True), C, M=M, N=N, K=K, x3=True)
    assert rel(C, A.double() @ Wt.double()) < TOL
    C0 = torch.randn(M, N, generator=g)
    C = C0.to(DEV)
    rgemm(A.to(DEV), Wx, C, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C, x3=True)
    assert rel(C, prod + C0.double()) < TOL
    src = torch.randn(M, N, generator=g)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), Wx, C, M=M, N=N, K=K, aux_mode=AUX_MASK, aux=src.to(DEV), aux_scale=1.25, x3=True)
    assert rel(C, torch.where(src.double() > 0, prod * 1.25, torch.zeros_like(prod))) < TOL
    keep = torch.nonzero(torch.rand(M, generator=g) < 0.6).reshape(-1)
    inv = torch.full((M,), -1, dtype=torch.int32)
    inv[keep] = torch.arange(keep.numel(), dtype=torch.int32)
    park = torch.randn(keep.numel(), N, generator=g)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), Wx, C, M=M, N=N, K=K, aux_mode=AUX_ACC_MAP, aux=park.to(DEV), auxmap=inv.to(DEV), x3=True)
    full = torch.zeros(M, N, dtype=torch.float64)
    full[keep] = park.double()
    assert rel(C, prod + full) < TOL


def test_rgemm_x3_relu_dropout_epilogue():
    from c2dsr_amd.ops import rgemm, to_split_bf16
    from oracle.c2dsr_oracle import keep_mask
    import numpy as np
    M, N, K, p = 333, 256, 256, 0.3
    g = torch.Generator().manual_seed(3)
    A, W, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g), torch.randn(N, generator=g)
    keys = (123456, 987654)
    C = torch.empty(M, N, device=DEV)
    rgemm(A.to(DEV), to_split_bf16(W.to(DEV)), C, M=M, N=N, K=K, bias=b.to(DEV), relu_drop=(keys, p, 1000), x3=True)
    idx = (np.arange(M)[:, None] + 1000) * N + np.arange(N)[None, :]
    mk = torch.from_numpy(keep_mask(idx, keys, p).astype(np.float32)).double() / (1 - p)
    ref = torch.relu(A.double() @ W.double().T + b.double()) * mk
    assert rel(C, ref) < TOL


@pytest.mark.parametrize('M,rowmap', [(4099, False), (1000, True), (57000, False), (40000, True)])
def test_rgemm_x3_relu_guard_signs(M, rowmap):
    """linear1 of the fp32 mode (c2dsr_rgemm_x3_relu_guard): split products with every pre-activation within
    the split error bound of zero recomputed exactly.  Inputs are built so that one column per row has a
    pre-activation ~1e-6 of ‖a‖‖w‖ (far inside the split error, outside fp32's): every ReLU decision with
    |v| > 2e-7·‖a‖‖w‖ matches float64 (the unguarded split product flips some of them), values within the
    fp32-mode tolerance, relu·dropout with the row map as c2dsr_rgemm's epilogue."""
    import numpy as np
    from c2dsr_amd.ops import rgemm, rgemm_relu_guard, to_split_bf16
    from oracle.c2dsr_oracle import keep_mask
    N, K, p = 256, 256, 0.2
    g = torch.Generator().manual_seed(M)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) / 16
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    b = torch.zeros(N, dtype=torch.float64)
    c = torch.arange(M) % N
    w = W[c]
    eps = (torch.rand(M, generator=g, dtype=torch.float64) - 0.5) * 2e-6
    A = A - ((A * w).sum(1) / (w * w).sum(1) - eps * A.norm(dim=1) / w.norm(dim=1))[:, None] * w
    A32, W32 = A.float(), W.float()
    v = A32.double() @ W32.double().T  # the fp32 operands' exact pre-activations
    scale = A32.double().norm(dim=1)[:, None] * W32.double().norm(dim=1)[None, :]
    keys = (2024, 77)
    rmap = torch.randperm(3 * M, generator=g)[:M].sort()[0].to(torch.int32) if rowmap else None
    rd = (keys, p, 500) + ((rmap.to(DEV),) if rowmap else ())
    rows = (rmap.numpy().astype(np.int64) if rowmap else np.arange(M)) + 500
    mk = torch.from_numpy(keep_mask(rows[:, None] * N + np.arange(N)[None, :], keys, p).astype(np.float32)).double()
    ref = torch.relu(v) * mk / (1 - p)
    Wx = to_split_bf16(W32.to(DEV))
    C = torch.empty(M, N, device=DEV)
    rgemm_relu_guard(A32.to(DEV), Wx, W32.to(DEV), C, M=M, N=N, K=K, bias=b.float().to(DEV), relu_drop=rd)
    C0 = torch.empty(M, N, device=DEV)
    rgemm(A32.to(DEV), Wx, C0, M=M, N=N, K=K, bias=b.float().to(DEV), relu_drop=rd, x3=True)
    Cf = torch.empty(M, N, device=DEV)  # the fragment-ordered image the training step uses: bit-identical
    rgemm_relu_guard(A32.to(DEV), to_split_bf16(W32.to(DEV), frag=True), W32.to(DEV), Cf, M=M, N=N, K=K,
                     bias=b.float().to(DEV), relu_drop=rd, frag=True)
    torch.cuda.synchronize()
    assert torch.equal(C, Cf)
    clear = (v.abs() > 2e-7 * scale) & (mk > 0)
    got, plain = C.double().cpu(), C0.double().cpu()
    assert torch.equal((got > 0)[clear], (v > 0)[clear])
    flips = int(((plain > 0) != (v > 0))[clear].sum())
    assert flips > 0, 'the inputs should put some pre-activations inside the split error'
    assert rel(C, ref) < TOL


@pytest.mark.parametrize('T,N', [(1000, 256), (4097, 768), (31, 128)])
def test_wgemm_x3_matches_float64(T, N):
    """Split-bf16 weight gradient dW = beta·dW + dYᵀ·X (+ exact fp32 bias sums) vs float64; deterministic;
    the multi-segment form (ops.WGradBatch) on ragged segments."""
    import numpy as np
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import wgemm
    D = 256
    g = torch.Generator().manual_seed(T + N)
    dY, X, W0 = torch.randn(T, N, generator=g), torch.randn(T, D, generator=g), torch.randn(N, D, generator=g)
    dW = W0.to(DEV)
    db = torch.full((N,), 3.0, device=DEV)
    wgemm(dY.to(DEV), X.to(DEV), dW, T=T, N=N, D=D, beta=1.0, db=db, x3=True)
    assert rel(dW, W0.double() + dY.double().T @ X.double()) < TOL
    assert rel(db, 3.0 + dY.double().sum(0)) < 1e-6
    dW2 = W0.to(DEV)
    wgemm(dY.to(DEV), X.to(DEV), dW2, T=T, N=N, D=D, beta=1.0, db=torch.full((N,), 3.0, device=DEV), x3=True)
    assert torch.equal(dW, dW2)
    Ts = (T, 33)
    dYs = [dY, torch.randn(33, N, generator=g)]
    Xs = [X, torch.randn(33, D, generator=g)]
    dYd, Xd = [y.to(DEV) for y in dYs], [x.to(DEV) for x in Xs]
    ws = torch.empty(lib.raw('c2dsr_wgemm_workspace')(N), dtype=torch.uint8, device=DEV)
    desc = np.asarray([v for y, x, t in zip(dYd, Xd, Ts) for v in (y.data_ptr(), N, x.data_ptr(), D, t)],
                      dtype=np.int64)
    dWm = torch.full((N, D), 0.5, device=DEV)
    lib('c2dsr_wgemm_x3_multi', desc, 2, N, D, 1.0, dWm, None, ws, stream())
    torch.cuda.synchronize()
    assert rel(dWm, 0.5 + sum(y.double().T @ x.double() for y, x in zip(dYs, Xs))) < TOL


def test_split_weight_images_multi():
    """c2dsr_to_split_bf16_multi (the optimizer-step refresh of the fp32 mode's weight images): both
    orientations equal the single conversions."""
    import numpy as np
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import to_split_bf16
    g = torch.Generator().manual_seed(9)
    Ws = [torch.randn(768, 256, generator=g).to(DEV), torch.randn(256, 256, generator=g).to(DEV)]
    outs, recs = [], []
    for W, tr in ((Ws[0], 0), (Ws[0], 1), (Ws[1], 1)):
        R, C = W.shape
        y = torch.empty((C, 2 * R) if tr else (R, 2 * C), device=DEV, dtype=torch.bfloat16)
        outs.append((y, to_split_bf16(W, bool(tr))))
        recs += [W.data_ptr(), y.data_ptr(), R, C, W.stride(0), tr]
    desc = np.asarray(recs, dtype=np.int64)
    lib('c2dsr_to_split_bf16_multi', desc, 3, stream())
    torch.cuda.synchronize()
    for y, ref in outs:
        assert torch.equal(y, ref)
    hi, lo = outs[1][1][:, :768].float(), outs[1][1][:, 768:].float()
    assert float((hi + lo - Ws[0].T).abs().max() / Ws[0].abs().max()) < 2 ** -16


def frag_index(n, k, hl, K):
    """c2dsr_to_split_bf16_frag_multi's element position (include/c2dsr.h), restated."""
    return (((n // 16) * (K // 16) + 2 * (k // 32) + hl) * 64 + ((k // 8) % 4) * 16 + n % 16) * 8 + k % 8


@pytest.mark.parametrize('N,K,tr', [(256, 256, 0), (768, 256, 0), (256, 512, 1), (200, 256, 0)])
def test_rgemm_x3_fragment_image(N, K, tr):
    """The fragment-ordered split image (c2dsr_to_split_bf16_frag_multi) is the row image's values at the header's
    positions, and c2dsr_rgemm_x3f on it is bit-identical to c2dsr_rgemm_x3 on the row image in every epilogue mode
    (the weight loads differ, the MFMA operands do not)."""
    from c2dsr_amd.ops import AUX_ACC, AUX_MASK, rgemm, to_split_bf16
    g = torch.Generator().manual_seed(N + K + tr)
    W = torch.randn(K, N, generator=g) if tr else torch.randn(N, K, generator=g)
    row = to_split_bf16(W.to(DEV), bool(tr)).cpu()
    frag = to_split_bf16(W.to(DEV), bool(tr), frag=True).cpu()
    assert frag.shape == (-(-N // 16) * 16, 2 * K)
    n, k = torch.meshgrid(torch.arange(N), torch.arange(K), indexing='ij')
    flat = frag.reshape(-1)
    for hl in (0, 1):
        assert torch.equal(flat[frag_index(n, k, hl, K)], row[:, hl * K:(hl + 1) * K])
    M = 1000 + 37
    A = torch.randn(M, K, generator=g).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    aux = torch.randn(M, N, generator=g).to(DEV)
    for kw in (dict(bias=b), dict(bias=b, relu_drop=((5, 6), 0.2, 100)), dict(aux_mode=AUX_MASK, aux=aux, aux_scale=2.0)):
        outs = []
        for fr, img in ((False, row.to(DEV)), (True, frag.to(DEV))):
            C = torch.empty(M, N, device=DEV)
            rgemm(A, img, C, M=M, N=N, K=K, x3=True, frag=fr, **kw)
            outs.append(C)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
    C0, C1 = aux.clone(), aux.clone()
    rgemm(A, row.to(DEV), C0, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C0, x3=True)
    rgemm(A, frag.to(DEV), C1, M=M, N=N, K=K, aux_mode=AUX_ACC, aux=C1, x3=True, frag=True)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)


def b16_frag_index(n, k, K):
    """c2dsr_to_bf16_frag_multi's element position (include/c2dsr.h), restated."""
    return (((n // 32) * (K // 16) + k // 16) * 64 + ((k // 8) % 2) * 32 + n % 32) * 8 + k % 8


@pytest.mark.parametrize('N,K,tr', [(256, 256, 0), (768, 256, 0), (256, 768, 1), (200, 512, 0)])
def test_rgemm_b16_fragment_image(N, K, tr):
    """The bf16 mode's weight image in fragment order (c2dsr_to_bf16_frag_multi, ops.weight_img 'b16') holds the
    row image's values at the header's positions, and the bf16 row-streaming kernel on it (ldb = 0) is bit-identical
    to the row image's in every epilogue mode, also with bf16 A (c2dsr_rgemm_aux_b16a, K = 768)."""
    import numpy as np
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import AUX_ACC, AUX_MASK, rgemm, to_bf16
    g = torch.Generator().manual_seed(N * 3 + K + tr)
    W = (torch.randn(K, N, generator=g) if tr else torch.randn(N, K, generator=g)).to(DEV)
    row = to_bf16(W, bool(tr))
    R, C = W.shape
    frag = torch.zeros(-(-N // 32) * 32, K, device=DEV, dtype=torch.bfloat16)
    desc = np.asarray([W.data_ptr(), frag.data_ptr(), R, C, W.stride(0), tr], dtype=np.int64)
    lib('c2dsr_to_bf16_frag_multi', desc, 1, stream())
    torch.cuda.synchronize()
    n, k = torch.meshgrid(torch.arange(N), torch.arange(K), indexing='ij')
    assert torch.equal(frag.cpu().reshape(-1)[b16_frag_index(n, k, K)], row.cpu())
    M = 1000 + 37
    A = torch.randn(M, K, generator=g).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    aux = torch.randn(M, N, generator=g).to(DEV)
    modes = [dict(bias=b), dict(aux_mode=AUX_ACC, aux=aux)]
    if K == 256:
        modes += [dict(bias=b, relu_drop=((5, 6), 0.2, 100)), dict(aux_mode=AUX_MASK, aux=aux, aux_scale=2.0)]
    for kw in modes:
        outs = []
        for fr, img in ((False, row), (True, frag)):
            Cm = torch.empty(M, N, device=DEV)
            rgemm(A, img, Cm, M=M, N=N, K=K, frag=fr, **kw)
            outs.append(Cm)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])
    if K == 768:  # bf16 A (the attention backward's dqkv)
        Ab = A.to(torch.bfloat16)
        outs = []
        for fr, img in ((False, row), (True, frag)):
            Cm = torch.empty(M, N, device=DEV)
            rgemm(Ab, img, Cm, M=M, N=N, K=K, frag=fr)
            outs.append(Cm)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])


def _ref_chunked(H, W, b, pl, t, coef, lam, BR, chunk=2048):
    """_ref in float64 on the device, in row chunks (the MB head-b logits are 9.7 GB in float64)."""
    H, W, b, pl, t = (x.to(DEV) for x in (H, W, b, pl, t))
    Hd, Wd, bd = H.double(), W.double(), b.double()
    M, n = H.shape[0], W.shape[0]
    lse = torch.empty(M, dtype=torch.float64, device=DEV)
    rows = torch.empty(M, dtype=torch.float64, device=DEV)
    dH = torch.empty(M, H.shape[1], dtype=torch.float64, device=DEV)
    gW = torch.zeros(n, H.shape[1], dtype=torch.float64, device=DEV)
    gb = torch.zeros(n, dtype=torch.float64, device=DEV)
    dpad = torch.empty(M, dtype=torch.float64, device=DEV)
    cf = coef.double().to(DEV)
    for r0 in range(0, M, chunk):
        r1 = min(M, r0 + chunk)
        lg = torch.cat([Hd[r0:r1] @ Wd.T + bd, pl[r0:r1].double()[:, None]], 1)
        ls = torch.logsumexp(lg, 1)
        tt = t[r0:r1]
        valid = tt != n
        lse[r0:r1] = ls
        rows[r0:r1] = torch.where(valid, ls - lg.gather(1, tt[:, None])[:, 0], torch.zeros_like(ls))
        w_r = torch.where(valid, lam * cf[(torch.arange(r0, r1, device=DEV) >= BR).long()], torch.zeros_like(ls))
        dl = torch.exp(lg - ls[:, None])
        dl[torch.arange(r1 - r0, device=DEV), tt] -= 1.0
        dl *= w_r[:, None]
        dH[r0:r1] = dl[:, :n] @ Wd
        gW += dl[:, :n].T @ Hd[r0:r1]
        gb += dl[:, :n].sum(0)
        dpad[r0:r1] = dl[:, n]
        del lg, dl
    return lse, rows, dH, gW, gb, dpad


def _shipped_dw(n, M, x3, D):
    """The dW sweep the loss head runs at this shape (losshead.dw_plan) in _run's convention: -1 stream-K, 0 one
    split added onto the gradients, k > 1 row splits summed."""
    from c2dsr_amd.losshead import dw_plan
    p = dw_plan(n, M, x3, D)
    return -1 if p == 0 else (0 if p == 1 else p)  # (p < 0: the remainder split, the same convention)


def test_ce3_mb_head_b_shape_matches_float64():
    """K5 at the headline's own shape: Movie-Book head b — Mv = 18,944 valid stacked rows,
    n = 63,937 columns, d = 256 — with the split counts losshead.py derives for it (split_count over 128-row /
    128-column tiles) and the XCD block map over ~2,000 column tiles, against float64 on the same fp32
    operands: full lse and per-row losses, the whole dH, dW and db.  Operand scales as in training: H like a
    LayerNorm output (unit normal), W / b like the classifier's nn.Linear init (U(±1/√d))."""
    from c2dsr_amd.losshead import split_count
    M, n, D = 18944, 63937, 256
    nr = _shipped_dw(n, M, True, D)
    g = torch.Generator().manual_seed(2048)
    H = torch.randn(M, D, generator=g)
    W = (torch.rand(n, D, generator=g) * 2 - 1) / 16
    b = (torch.rand(n, generator=g) * 2 - 1) / 16
    pl = torch.randn(M, generator=g) * 0.3
    t = torch.randint(0, n, (M,), generator=g)
    coef, lam, BR = torch.tensor([0.45, 1.0]), 0.7, 9100
    ns = split_count(M, 128)
    lse, rows, dH, gW, gb, dpad, _ = _run(H, W, b, pl, t, coef, lam, ns, nr, BR)
    ref = _ref_chunked(H, W, b, pl, t, coef, lam, BR)
    err = {k: rel(x, r) for k, x, r in zip(('lse', 'rows', 'dH', 'gW', 'gb', 'dpad'), (lse, rows, dH, gW, gb, dpad),
                                           ref)}
    print(f'ce3 MB head b (ns={ns}, nr={nr}) errors', {k: f'{v:.2e}' for k, v in err.items()})
    assert err.pop('lse') < TOL_LSE
    assert all(v < TOL for v in err.values()), err


def test_ce3b_mb_head_b_shape_matches_float64():
    """The bf16 mode's K5 (ce3b) at the same headline shape, on operands already representable in bf16 (H and W
    rounded once on the host), against float64 on those same operands.  The bf16 images are then exact, so the
    logits carry only fp32 accumulation error (lse / per-row losses to TOL_LSE / TOL); the gradient products
    take the softmax weights as bf16 (relative 2^-9 per term, unbiased rounding over n = 63,937 terms), held
    here to north_star's 1e-4 of their max-abs (measured: dH 2.3e-5, dW 2.7e-6, db 1.2e-7 — the end-to-end
    bf16 comparison's 7e-2 is dominated by the bf16 encoder, not K5)."""
    from c2dsr_amd.losshead import split_count
    M, n, D = 18944, 63937, 256
    nr = _shipped_dw(n, M, False, D)
    g = torch.Generator().manual_seed(4096)
    H = torch.randn(M, D, generator=g).bfloat16().float()
    W = ((torch.rand(n, D, generator=g) * 2 - 1) / 16).bfloat16().float()
    b = (torch.rand(n, generator=g) * 2 - 1) / 16
    pl = torch.randn(M, generator=g) * 0.3
    t = torch.randint(0, n, (M,), generator=g)
    coef, lam, BR = torch.tensor([0.45, 1.0]), 0.7, 9100
    ns = split_count(M, 128)
    lse, rows, dH, gW, gb, dpad, _ = _run(H, W, b, pl, t, coef, lam, ns, nr, BR, b16=True)
    ref = _ref_chunked(H, W, b, pl, t, coef, lam, BR)
    err = {k: rel(x, r) for k, x, r in zip(('lse', 'rows', 'dH', 'gW', 'gb', 'dpad'), (lse, rows, dH, gW, gb, dpad),
                                           ref)}
    print(f'ce3b MB head b (ns={ns}, nr={nr}) errors', {k: f'{v:.2e}' for k, v in err.items()})
    assert err.pop('lse') < TOL_LSE
    assert err.pop('rows') < TOL
    assert all(v < 1e-4 for v in err.values()), err


@pytest.mark.parametrize('M,n,D,ns', [(300, 700, 256, 3), (1000, 2100, 128, 4), (33, 31, 256, 2), (777, 4099, 256, 7)])
def test_ce3_stored_logits_layout(M, n, D, ns):
    """c2dsr_ce3_fused_fwd_u_lg's logits buffer read back through the layout include/c2dsr.h documents (16 × 16 blocks,
    column-block-major, element (r, c) at ((r%16)/4·16 + c%16)·4 + r%4): v = (h_r·w_c + b_c)·log2e for r < M, c < n
    (the fp32 mode's split products: within 1e-5 of max-abs), −inf for the padding columns c < ⌈n/32⌉·32, and the
    forward's other outputs equal to the plain sweep's bit for bit."""
    from c2dsr_amd._lib import lib, stream
    s = stream()
    g = torch.Generator().manual_seed(M * 3 + n)
    H = torch.randn(M, D, generator=g) * 0.5
    W = torch.randn(n, D, generator=g) * 0.5
    b = torch.randn(n, generator=g) * 0.1
    pl = torch.randn(M, generator=g)
    t = torch.randint(0, n + 1, (M,), generator=g)
    M_pad, n32, n_pad = max(64, -(-M // 64) * 64), -(-n // 32) * 32, -(-n // 128) * 128 + 64
    Hx = torch.empty(M_pad, 2 * D, dtype=torch.bfloat16, device=DEV)
    Wx = torch.empty(n32, 2 * D, dtype=torch.bfloat16, device=DEV)
    lib('c2dsr_f32_split_bf16', H.to(DEV), M, D, M_pad, Hx, s)
    lib('c2dsr_f32_split_bf16', W.to(DEV), n, D, n32, Wx, s)
    bias2 = torch.empty(n_pad, device=DEV)
    lib('c2dsr_ce_bias2', b.to(DEV), n, n_pad, bias2, s)
    outs = []
    for use_lg in (False, True):
        o = [torch.empty(ns, M, device=DEV), torch.empty(ns, M, device=DEV), torch.empty(ns, M, D, device=DEV),
             torch.empty(M, device=DEV), torch.empty(M_pad, device=DEV), torch.empty(M, device=DEV)]
        a = (Hx, Wx, bias2, M, n, D, ns, o[0], o[1], o[2], pl.to(DEV), t.to(DEV), H.to(DEV), W.to(DEV), b.to(DEV),
             o[3], o[4], o[5])
        if use_lg:
            lg = torch.full((int(lib.raw('c2dsr_ce3_logits_floats')(M, n)),), float('nan'), device=DEV)
            lib('c2dsr_ce3_fused_fwd_u_lg', *a, lg, s)
        else:
            lib('c2dsr_ce3_fused_fwd_u', *a, s)
        outs.append(o)
    torch.cuda.synchronize()
    for x, y in zip(*outs):
        assert torch.equal(x[..., :M] if x.dim() == 1 else x, y[..., :M] if y.dim() == 1 else y)
    HB = -(-M // 128) * 8
    grp = int(lib.raw('c2dsr_ce3_logits_group')(0))
    CW = -(-(n32 // 16) // grp) * grp
    assert lg.numel() == CW * HB * 256
    # [c/16/grp][r/16][(c/16)%grp][(r%16)/4][c%16][r%4]
    blk = lg.cpu().view(CW // grp, HB, grp, 4, 16, 4)
    full = blk.permute(1, 3, 5, 0, 2, 4).reshape(HB * 16, CW * 16)  # [r][c]
    ref = (H.double() @ W.double().T + b.double()) * 1.4426950408889634
    got = full[:M, :n].double()
    err = float((got - ref).abs().max() / ref.abs().max())
    print('stored logits rel err', err)
    assert err < 1e-5
    assert bool(torch.isneginf(full[:M, n:n32]).all())
