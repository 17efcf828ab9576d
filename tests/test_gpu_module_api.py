"""The reference's module API, called directly with reference-typed arguments (SURVEY.md §8(b);
models/C2DSR.py:9-85, models/encoders.py:7-48): ``C2DSR(args, adj, adj_specific)`` built from the torch
sparse COO adjacency ``utils/graph.make_graph`` returns, then ``convolve_graph``, ``forward``,
``forward_share``, ``GCN.forward(h, adj) -> [N, d]`` and ``SelfAttention.forward(seq, seq_enc, pos)`` (which
mutates ``seq_enc`` in place, Q20) against the intermediates the reference itself produced on the same
parameters and batch (tests/golden/model_*.npz, tools/gen_fixtures.py; dropout 0, fp32 mode, 1e-4)."""
import math

import pytest
import torch
import torch.nn.functional as F

from tests import goldens as G
from tests.test_gpu_parity import make_args, rel

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL = 1e-4


def coo(name, kind, n):
    """The adjacency exactly as utils/graph.py:20-26 hands it to the model: torch sparse COO [n, n], fp32."""
    g = G.load(f'graph_{name}.npz')
    idx = torch.stack([torch.from_numpy(g[f'{kind}_row']), torch.from_numpy(g[f'{kind}_col'])]).long()
    return torch.sparse_coo_tensor(idx, torch.from_numpy(g[f'{kind}_val']).float(), (n, n)).to(DEV)


def build(name):
    from c2dsr_amd.models.C2DSR import C2DSR
    c = G.CONFIGS[name]
    args = make_args(c)
    n = c['n_a'] + c['n_b'] + 1
    adj_s, adj_p = coo(name, 'share', n), coo(name, 'specific', n)
    model = C2DSR(args, adj_s, adj_p).to(DEV)
    P = G.init_params(name)
    with torch.no_grad():
        for k, p in model.named_parameters():
            if k in P:
                p.copy_(P[k].to(DEV))
    model.train()  # dropout 0: the reference's training-mode forward, deterministic
    return model, adj_s, adj_p, c


@pytest.mark.parametrize('name', ['base', 'var', 'shared'])
def test_module_api_matches_reference_intermediates(name):
    model, adj_s, adj_p, c = build(name)
    m = G.load(f'model_{name}.npz')
    d = c['d_latent']
    model.convolve_graph()
    for k in ('hi_share', 'hi_a', 'hi_b'):
        assert rel(getattr(model, k), m[f's0/{k}']) < TOL, k
    # GCN.forward(h, adj) on the reference's sparse COO → [N, d]
    for gnn, E, adj, k in ((model.gnn_share, model.embed_i.weight, adj_s, 'hi_share'),
                           (model.gnn_a, model.embed_i_a.weight, adj_p, 'hi_a')):
        H = gnn(E, adj)
        assert isinstance(H, torch.Tensor) and H.shape == E.shape
        assert rel(H, m[f's0/{k}']) < TOL, k
    b = [x.to(DEV) for x in G.batch(name, int(m['s0/batch_lo']), int(m['s0/batch_n']))]
    seq_share, seq_a, seq_b, pos, pos_a, pos_b = b[:6]
    neg_a, neg_b = b[12], b[13]
    h_share, hx, hy = model(seq_share, seq_a, seq_b, pos, pos_a, pos_b)
    for got, k in ((h_share, 'h_share'), (hx, 'hx'), (hy, 'hy')):
        assert got.shape == tuple(m[f's0/{k}'].shape) and rel(got, m[f's0/{k}']) < TOL, k
    assert rel(model.forward_share(neg_a, pos), m['s0/h_neg_a']) < TOL
    assert rel(model.forward_share(neg_b, pos), m['s0/h_neg_b']) < TOL
    # SelfAttention.forward on a caller-built seq_enc (C2DSR.py:65-71), mutated in place (encoders.py:30)
    with torch.no_grad():
        enc = (F.embedding(seq_share, model.hi_share) + model.embed_i.weight[seq_share]) * math.sqrt(d)
    before = enc.clone()
    out = model.attn_share(seq_share, enc, pos)
    assert rel(out, m['s0/h_share']) < TOL
    want = before + model.attn_share.pos_emb.weight.detach()[pos]
    assert torch.allclose(enc, want, rtol=0, atol=1e-6), 'seq_enc must hold seq_enc + pos_emb(pos) (Q20)'


@pytest.mark.parametrize('name', ['base', 'var'])
def test_gcn_module_backward_vs_dense(name):
    """GCN.forward's gradient w.r.t. h (dropout 0): Σ_k (Aᵀ)^k R / (n_gnn + 1) for R = dL/dH, against the
    dense adjacency on the device."""
    model, adj_s, _, c = build(name)
    E = model.embed_i.weight.detach().clone().requires_grad_(True)
    H = model.gnn_share(E, adj_s)
    R = torch.randn(H.shape, generator=torch.Generator().manual_seed(3)).to(DEV)
    (H * R).sum().backward()
    A = adj_s.to_dense().double()
    n = c['n_gnn']
    t, ref = R.double(), R.double().clone()
    for _ in range(n):
        t = A.T @ t
        ref += t
    ref /= n + 1
    assert rel(E.grad, ref) < 1e-5
    hf = E.detach().double()
    Hr, acc = hf.clone(), hf.clone()
    for _ in range(n):
        acc = A @ acc
        Hr += acc
    assert rel(H, Hr / (n + 1)) < 1e-5


def test_self_attention_inplace_autograd():
    """The in-place position add is an autograd-visible in-place op: a caller that also uses the mutated
    seq_enc gets the sum of both gradients on the original values."""
    model, _, _, c = build('base')
    d, L = c['d_latent'], c['len_max']
    b = [x.to(DEV) for x in G.batch('base', 0, 16)]
    seq, pos = b[0], b[3]
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(16, L, d, generator=g).to(DEV).requires_grad_(True)
    R2 = torch.randn(16, L, d, generator=g).to(DEV)
    enc = x0 * 1.0
    out = model.attn_share(seq, enc, pos)
    (out.sum() + (enc * R2).sum()).backward()
    x1 = x0.detach().clone().requires_grad_(True)
    out1 = model.attn_share(seq, x1 * 1.0, pos)
    out1.sum().backward()
    assert rel(out, out1) < 1e-6
    assert rel(x0.grad, x1.grad + R2) < 1e-5
