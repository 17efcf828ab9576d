"""Evaluation path on the device (csrc/eval.hip via Trainer.evaluate_batch /
run_epoch / run_test / evaluate_metrics) against the reference's golden ranks and metrics.
Ranks are integer results: bit-exact against the fixtures; at large synthetic sizes the check is
tie-robust (rank within the fp64 bounds of a ±1e-5 relative score band)."""
import numpy as np
import pytest
import torch

from tests import goldens as G
from tests.test_gpu_parity import build_trainer, golden_graphs, make_args

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _eval_batch(name, mode):
    d = G.load(f'data_{name}.npz')
    return tuple(torch.from_numpy(np.ascontiguousarray(d[f'{mode}_{j}'])) for j in range(11))


def _eval_trainer(name):
    e = G.load(f'eval_{name}.npz')
    params = {k[len('param/'):]: torch.from_numpy(e[k].copy()) for k in e.files if k.startswith('param/')}
    gs, gp = golden_graphs(name)
    return build_trainer(make_args(G.CONFIGS[name]), gs, gp, params), e


@pytest.mark.parametrize('name', list(G.CONFIGS))
def test_eval_ranks_match_reference(name):
    tr, e = _eval_trainer(name)
    tr.model.eval()
    with torch.no_grad():
        tr.model.convolve_graph()
        for mode in ('val', 'test'):
            b = _eval_batch(name, mode)
            ra, rb = tr.evaluate_batch(b)
            assert ra == e[f'{mode}_rank_a'].tolist(), (mode, 'a')
            assert rb == e[f'{mode}_rank_b'].tolist(), (mode, 'b')
            # the multi-batch pass (one host sync) gives the same lists
            half = b[0].shape[0] // 2
            parts = [tuple(x[:half] for x in b), tuple(x[half:] for x in b)]
            assert tr._evaluate(parts) == (ra, rb)


def test_device_metrics_match_reference():
    from c2dsr_amd.metrics import RankMetrics
    m = G.load('metrics.npz')
    ra, rb = m['ranks_a'], m['ranks_b']
    rank = torch.tensor(np.concatenate([ra, rb]), dtype=torch.int32, device=DEV)
    xory = torch.tensor([0] * len(ra) + [1] * len(rb), dtype=torch.int64, device=DEV)
    acc = RankMetrics(DEV)
    acc.add(rank[:50], xory[:50])  # accumulation over batches
    acc.add(rank[50:], xory[50:])
    ma, _ = acc.values()
    np.testing.assert_allclose(ma, m['metrics_a'], rtol=1e-12)
    np.testing.assert_allclose(acc.score([0.1124, 0.0865, 0.0574, 0.0416]), m['score_fk'], rtol=1e-12)
    np.testing.assert_allclose(acc.score([0.0647, 0.0476, 0.0284, 0.0217]), m['score_mb'], rtol=1e-12)


@pytest.mark.parametrize('d,n_neg,L', [(256, 999, 50), (64, 999, 15), (16, 10, 8), (30, 37, 5)])
def test_eval_rank_kernel_large(d, n_neg, L):
    """Synthetic rows at the metric's sizes (d=256, 999 negatives): ranks vs fp64 scores, with the
    target planted among the negatives (an equal score is not counted)."""
    from c2dsr_amd import ops
    g = torch.Generator().manual_seed(d + n_neg)
    B, n_a, n_b = 300, 5000, 7000
    hs, ha, hb = (torch.randn(B, L, d, generator=g) for _ in range(3))
    Wa, Wb = torch.randn(n_a, d, generator=g) * 0.1, torch.randn(n_b, d, generator=g) * 0.1
    ba, bb = torch.randn(n_a, generator=g), torch.randn(n_b, generator=g)
    xory = torch.randint(0, 2, (B, 1), generator=g)
    il_a, il_b = torch.randint(0, L, (B, 1), generator=g), torch.randint(0, L, (B, 1), generator=g)
    # no prior item in the domain: the reference reads hx[i, -1] (Python wrap to L-1)
    il_a[::5], il_b[::7], il_b[1::11] = -1, -1, -L
    n_dom = torch.where(xory[:, 0] == 0, n_a, n_b)
    gt = (torch.rand(B, 1, generator=g) * n_dom[:, None]).long()
    neg = (torch.rand(B, n_neg, generator=g) * n_dom[:, None]).long()
    neg[::3, 0] = gt[::3, 0]
    neg[1::13, 1] = -1  # torch indexing wraps a negative item id too (scores[-1])
    got = ops.eval_rank(*(t.to(DEV) for t in (hs, ha, hb, il_a, il_b, xory, gt, neg, Wa, ba, Wb, bb))).cpu()
    for i in range(B):
        dom_a = int(xory[i]) == 0
        q = (hs[i, -1] + (ha if dom_a else hb)[i, int((il_a if dom_a else il_b)[i])]).double()
        W, b = (Wa, ba) if dom_a else (Wb, bb)
        s = W.double() @ q + b.double()
        sg = s[gt[i, 0]]
        sn = s[neg[i]]  # wraps negative ids like the reference's scores_a[list_neg[i]]
        band = 1e-5 * float(s.abs().max())
        lo = 1 + int((sn > sg + band).sum())
        same = (neg[i] % len(s)) == (gt[i, 0] % len(s))
        hi = 1 + int(((sn > sg - band) & ~same).sum())
        assert lo <= int(got[i]) <= hi, (i, int(got[i]), lo, hi)


def test_eval_rank_bad_index_raises():
    tr, _ = _eval_trainer('base')
    b = list(_eval_batch('base', 'val'))
    b[10] = b[10].clone()
    b[10][0, 0] = 10 ** 6  # negative item id out of range
    tr.model.eval()
    with torch.no_grad():
        tr.model.convolve_graph()
        with pytest.raises(IndexError):
            tr.evaluate_batch(tuple(b))
