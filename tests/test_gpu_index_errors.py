"""The reference's "bad input raises" contract on the training path.

The reference's lookups raise IndexError for an index outside their table — F.embedding(seq, hi_*) /
nn.Embedding(seq) (models/C2DSR.py:65-67,81), pos_emb(pos) (models/encoders.py:30), F.cross_entropy on a target
outside [0, n] other than the ignore index (trainer.py:143-152) — inside the forward, so nothing is updated.  Here:
  * a batch with a host copy is checked on the host before anything is enqueued (Trainer.check_batch_indices);
  * a device batch without one is range-checked on the device (c2dsr::index_check) and the verdict rides on the
    step's deferred count read, which raises in the forward, before any backward or optimizer launch;
  * underneath, every lookup kernel range-checks its own indices into the device error word and reads row 0
    instead, the index plans sort a bad key past every table row so no segment sum follows it, and AdamW changes
    nothing while the word is set (include/c2dsr.h C2DSR_IDX_ERR_*).
"""
import math

import numpy as np
import pytest
import torch

from tests import goldens as G
from tests.test_gpu_parity import DEV, build_trainer, golden_graphs, make_args, rel

pytestmark = pytest.mark.gpu


def _trainer(name='base'):
    gs, gp = golden_graphs(name)
    tr = build_trainer(make_args(G.CONFIGS[name]), gs, gp, G.init_params(name))
    tr.model.train()
    tr.optimizer.zero_grad()
    return tr


def _state(tr):
    f = tr.model.flat
    return f.param.clone(), f.accum.clone(), tr.optimizer  # (optimizer kept for its step count)


def _bad(batch, k, row, col, v):
    out = [t.clone() for t in batch]
    out[k][row, col] = v
    return tuple(out)


CASES = [(0, 'n_item', 'item index'), (12, 'n_item', 'item index'), (2, -1, 'item index'),
         (3, 'len_max', 'position'), (6, 'n_a+1', 'target')]


def _value(tr, v):
    c = G.CONFIGS['base']
    return {'n_item': tr.model.n_item, 'len_max': c['len_max'], 'n_a+1': c['n_a'] + 1}.get(v, v)


@pytest.mark.parametrize('k,v,what', CASES)
@pytest.mark.parametrize('where', ['host', 'device'])
def test_out_of_range_index_raises_and_changes_nothing(k, v, what, where):
    tr = _trainer()
    b = G.batch('base', 0, 16)
    L = b[0].shape[1]
    bad = _bad(b, k, 5, L - 1, _value(tr, v))
    if where == 'device':
        bad = tuple(t.to(DEV) for t in bad)  # no host copy: the device check decides
    tr.model.convolve_graph()
    torch.cuda.synchronize()
    p0, a0, _ = _state(tr)
    with pytest.raises(IndexError, match=what):
        tr.train_batch(bad)
    torch.cuda.synchronize()
    assert torch.equal(tr.model.flat.param, p0), 'parameters changed by a step that raised'
    assert torch.equal(tr.model.flat.accum, a0), 'gradient tables changed by a step that raised'
    assert int(torch.ops.c2dsr.error_word()[0]) == 0, 'the raise clears the error word'
    # the trainer is usable afterwards: the next (valid) step is the reference's golden step 0
    m = G.load('model_base.npz')
    tr.model.convolve_graph()
    loss, _, _ = tr.train_batch(b)
    assert abs(float(loss.detach()) - float(m['s0/loss'])) <= 1e-4 * abs(float(m['s0/loss']))
    assert rel(tr.model.flat.grad_total('classifier_a.weight'), m['s0/grad/classifier_a.weight']) < 1e-4


def test_device_flags_without_precheck_skip_adamw_and_raise_at_epoch_sync():
    """The kernels' own flags (no batch check at all: counts handed in, as a pipeline that skipped launch_counts
    would): the bad lookups read row 0, the bad key is never followed by the segment sums, AdamW changes nothing,
    and check_index_errors (run_epoch's sync) raises."""
    tr = _trainer()
    b = G.batch('base', 0, 16)
    L = b[0].shape[1]
    bad = _bad(b, 1, 3, L - 2, tr.model.n_item + 3)  # seq_a
    hb = tuple(np.asarray(x) for x in bad)  # counts straight from host_counts, which does not range-check
    need, pads, ce = tr.count_flags(L)
    counts = tr.host_counts(hb, need=need, pads=pads, ce=ce)
    tr.model.convolve_graph()
    torch.cuda.synchronize()
    p0 = tr.model.flat.param.clone()
    tr.train_batch(tuple(t.to(DEV) for t in bad), counts=counts)
    torch.cuda.synchronize()
    w = int(torch.ops.c2dsr.error_word()[0])
    assert w & 1, f'item-index bit not set ({w:#x})'
    assert torch.equal(tr.model.flat.param, p0), 'AdamW ran with the error word set'
    assert torch.isfinite(tr.model.flat.accum).all()
    with pytest.raises(IndexError, match='item index'):
        tr.check_index_errors()
    assert int(torch.ops.c2dsr.error_word()[0]) == 0
    tr.check_index_errors()  # cleared: nothing pending


def test_embed_kernels_clamp_and_flag():
    """Kernel level: the gather reads row 0 for a bad item index (no load leaves the table) and flags it; the index
    plan sorts a bad key past every row and the segment sums skip it; a valid key's sums are untouched."""
    from c2dsr_amd._lib import lib, stream
    rng = np.random.default_rng(11)
    n_items, L, d, B = 50, 10, 64, 40
    n = B * L
    seq = rng.integers(0, n_items, size=n)
    pos = rng.integers(0, L, size=n)
    seq[7], seq[100], pos[33] = n_items, -4, L + 2
    H, E, P = torch.randn(n_items, d), torch.randn(n_items, d), torch.randn(L, d)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    X = torch.empty(n, d, device=DEV)
    sd, pd = torch.from_numpy(seq).to(DEV), torch.from_numpy(pos).to(DEV)
    lib('c2dsr_embed_fwd', sd, pd, n, d, H.to(DEV), E.to(DEV), None, P.to(DEV), math.sqrt(d), 0, 0, 0.0, 0, X,
        n_items, L, err, stream())
    assert int(err[0]) == 1 | 2
    s_ok = np.where((seq >= 0) & (seq < n_items), seq, 0)
    p_ok = np.where((pos >= 0) & (pos < L), pos, 0)
    ref = (H[s_ok] + E[s_ok]) * math.sqrt(d) + P[p_ok]
    assert rel(X, ref) < 1e-6
    # backward over plans: the bad key contributes nowhere
    err.zero_()
    pb = int(lib.raw('c2dsr_index_plan_bytes')(n))
    sp = torch.empty(pb, dtype=torch.uint8, device=DEV)
    lib('c2dsr_index_plan', sd, n, n_items, sp, pb, err, stream())
    assert int(err[0]) == 4
    gX = torch.randn(n, d)
    Gt = torch.zeros(n_items + 8, d, device=DEV)  # rows past n_items: a canary for an out-of-table write
    ws_bytes = int(lib.raw('c2dsr_embed_bwd_planned_workspace')(n, d))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=DEV)
    lib('c2dsr_embed_bwd_planned', sp, None, n, d, gX.to(DEV), 0, 0, 0.0, 0, 1.0, Gt, n_items, None, 0, None, ws,
        ws_bytes, stream())
    want = torch.zeros(n_items + 8, d, dtype=torch.float64)
    for r in range(n):
        if 0 <= seq[r] < n_items:
            want[seq[r]] += gX[r].double()
    assert rel(Gt, want) < 1e-5
    assert float(Gt[n_items:].abs().max()) == 0.0


def test_adamw_changes_nothing_while_the_error_word_is_set():
    from c2dsr_amd._lib import lib, stream
    n = 4096
    bufs = [torch.randn(n, device=DEV) for _ in range(6)]
    before = [t.clone() for t in bufs]
    err = torch.tensor([2, 0, 0, 0], dtype=torch.int32, device=DEV)
    lib('c2dsr_adamw', *bufs, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, 1, err, stream())
    assert all(torch.equal(a, b) for a, b in zip(bufs, before))
    err.zero_()
    lib('c2dsr_adamw', *bufs, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, 1, err, stream())
    assert not torch.equal(bufs[0], before[0])


def test_compact_valid_flags_bad_targets():
    from c2dsr_amd._lib import lib, stream
    M, ignore = 3000, 99
    t = np.random.default_rng(5).integers(0, ignore + 1, M)
    t[17], t[2000] = ignore + 1, -3
    tt = torch.from_numpy(t).to(DEV)
    idx = torch.empty(M, device=DEV, dtype=torch.int32)
    inv = torch.empty(M, device=DEV, dtype=torch.int32)
    tc = torch.empty(M, device=DEV, dtype=torch.int64)
    cnt = torch.empty(2, device=DEV, dtype=torch.int32)
    ws = torch.empty(lib.raw('c2dsr_compact_workspace')(M, 1) // 4 + 1, device=DEV, dtype=torch.int32)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    lib('c2dsr_compact_valid', tt, M, M // 2, ignore, idx, inv, tc, cnt, ws, err, stream())
    assert int(err[0]) == 8
    valid = (t >= 0) & (t < ignore)
    assert int(cnt.sum()) == int(valid.sum())
    assert int(inv[17]) == -1 and int(inv[2000]) == -1


@pytest.mark.parametrize('n,n_keys,hot', [(102_400, 36_846, 0.45), (20_000, 50, 0.0), (5_000, 7, 0.9), (1, 3, 0.0),
                                          (300_001, 100_000, 0.6)])
def test_index_plan_structure(n, n_keys, hot):
    """The plan's sort, split list and SUBP-piece sub-ranges (built in plan_count / plan_emit since round 6 — the
    single-workgroup plan_subs launch is gone) against the host restatement ops._check_plan, with a hot key whose
    run spans far more than SUBP chunks, and out-of-range indices (sorted last as the key n_keys)."""
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import _check_plan
    rng = np.random.default_rng(n)
    x = rng.zipf(1.3, size=n) % n_keys
    x[rng.random(n) < hot] = n_keys - 1
    if n > 10:
        x[3], x[n // 2] = n_keys + 2, -1
    idx = torch.from_numpy(x.astype(np.int64)).to(DEV)
    pb = int(lib.raw('c2dsr_index_plan_bytes')(n))
    buf = torch.empty(pb, dtype=torch.uint8, device=DEV)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    lib('c2dsr_index_plan', idx, n, n_keys, buf, pb, err, stream())
    _check_plan(buf, idx, n_keys)
    assert int(err[0]) == (4 if n > 10 else 0)


def test_index_plans_batched_equal_single():
    """c2dsr_index_plans (one launch per pass over all the plans, as the training step builds its eight lookup plans)
    writes, plan by plan, exactly what c2dsr_index_plan writes for each alone: mixed key widths (1, 2 and 3 radix
    passes in one launch set), an out-of-range index, a hot key, an empty job, more jobs than one launch group."""
    from c2dsr_amd._lib import lib, stream
    from c2dsr_amd.ops import _check_plan
    rng = np.random.default_rng(7)
    jobs = []
    for k, (n, n_keys) in enumerate([(102_400, 36_846), (102_400, 51), (50_000, 64_000), (0, 10), (7, 3),
                                     (30_000, 300), (20_000, 2 ** 20), (102_400, 51), (1, 5), (4096, 4096),
                                     (9000, 100_000), (12_345, 70), (5000, 255), (5000, 256)]):
        x = (rng.zipf(1.3, size=n) % n_keys).astype(np.int64)
        if n > 100:
            x[rng.random(n) < 0.3] = n_keys - 1
            x[n // 3] = n_keys + 5 if k % 2 else -2
        jobs.append((torch.from_numpy(x).to(DEV), n, n_keys))
    sizes = [int(lib.raw('c2dsr_index_plan_bytes')(n)) if n else 256 for _, n, _ in jobs]
    single = [torch.zeros(s, dtype=torch.uint8, device=DEV) for s in sizes]
    multi = [torch.zeros(s, dtype=torch.uint8, device=DEV) for s in sizes]
    e1 = torch.zeros(4, dtype=torch.int32, device=DEV)
    e2 = torch.zeros(4, dtype=torch.int32, device=DEV)
    for (idx, n, nk), buf, s in zip(jobs, single, sizes):
        lib('c2dsr_index_plan', idx, n, nk, buf, s, e1, stream())
    desc = torch.tensor([[idx.data_ptr(), n, nk, buf.data_ptr(), s] for (idx, n, nk), buf, s in zip(jobs, multi, sizes)],
                        dtype=torch.int64)
    lib('c2dsr_index_plans', desc, len(jobs), e2, stream())
    torch.cuda.synchronize()
    assert int(e1[0]) == int(e2[0]) == 4
    for (idx, n, nk), a, b in zip(jobs, single, multi):
        if n == 0:
            continue
        _check_plan(b, idx, nk)
        # the bytes the consumers read (keys, rows, split list, counts, sub-ranges) are the single plan's
        assert torch.equal(a[:8 * n], b[:8 * n]), (n, nk)
        _check_plan(a, idx, nk)
