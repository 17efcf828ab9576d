"""The stage operators the training step runs on (c2dsr::encoder_pass / encoder_pass_backward, gcn_propagate /
gcn_backward_*, embed_fuse*, index_plans, adamw_step; csrc_torch/) against the op-by-op path they replace (the same
kernels launched one by one from c2dsr_amd/ops.py): two training steps at the benchmarked shape (d = 256, L = 50,
R = 10) with dropout 0.2, in both precision modes — the losses, every gradient and the updated parameters are
bit-identical.  Also: the fused pass and loss head are the ones taken."""
import numpy as np
import pytest
import torch

from tests.test_gpu_parity import build_trainer, capture, make_args

pytestmark = pytest.mark.gpu

C = dict(n_a=300, n_b=400, len_max=50, len_rec=10, d_latent=256, n_gnn=1, n_attn=1, n_head=1, norm_first=False,
         d_bias=False, shared_item_embed=False)


def _case(precision):
    import random
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import synth
    seqs = synth.make_sequences(300, C['n_a'], C['n_b'], C['len_max'], seed=3, n_min=6)
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, C['n_a'], C['n_b'], C['len_max']))
    gs, gp = GR.preprocess_graph(seqs, C['n_a'], C['n_a'] + C['n_b'] + 1)
    return rows, gs, gp


def _run(precision, fused, rows, gs, gp, B=96):
    from c2dsr_amd import losshead, ops
    ops.FUSED_PASS = losshead.FUSED_HEAD = fused
    try:
        args = make_args(C, dropout=0.2, precision=precision, seed=5)
        args.batch_size = B
        torch.manual_seed(1234)
        tr = build_trainer(args, gs, gp)
        tr.model.train()
        tr.optimizer.zero_grad()
        out = []
        for s in range(2):
            box = capture(tr)
            tr.model.convolve_graph()
            loss, loss_rec, loss_mi = tr.train_batch(tuple(torch.from_numpy(r[s * B:(s + 1) * B].copy()) for r in rows))
            torch.cuda.synchronize()
            out.append(dict(loss=[float(loss), float(loss_rec), float(loss_mi)], grads=box['grads']))
        params = {n: p.detach().cpu().clone() for n, p in tr.model.named_parameters()}
        return out, params
    finally:
        ops.FUSED_PASS = losshead.FUSED_HEAD = True


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_fused_pass_equals_op_by_op_path(precision):
    rows, gs, gp = _case(precision)
    a, pa = _run(precision, True, rows, gs, gp)
    b, pb = _run(precision, False, rows, gs, gp)
    for s, (x, y) in enumerate(zip(a, b)):
        assert x['loss'] == y['loss'], (s, x['loss'], y['loss'])
        for n in x['grads']:
            assert torch.equal(x['grads'][n], y['grads'][n]), (s, n)
    for n in pa:
        assert torch.equal(pa[n], pb[n]), n


def test_fused_pass_and_head_are_taken():
    """The fused pass runs (once per pass each way) and the loss head takes the stage operators."""
    from c2dsr_amd import losshead, ops
    rows, gs, gp = _case('fp32')
    args = make_args(C, dropout=0.2, precision='fp32', seed=5)
    args.batch_size = 96
    torch.manual_seed(1234)
    tr = build_trainer(args, gs, gp)
    tr.model.train()
    tr.optimizer.zero_grad()
    calls = {'fwd': 0, 'bwd': 0, 'head': 0}
    f0, b0 = ops.EncoderPassFn.forward, ops.EncoderPassFn.backward
    h0 = losshead.LossHeadFn._backward_stage

    def head(*a):
        calls['head'] += 1
        return h0(*a)

    def fwd(*a):
        calls['fwd'] += 1
        return f0(*a)

    def bwd(*a):
        calls['bwd'] += 1
        return b0(*a)
    ops.EncoderPassFn.forward, ops.EncoderPassFn.backward = staticmethod(fwd), staticmethod(bwd)
    losshead.LossHeadFn._backward_stage = staticmethod(head)
    try:
        tr.model.convolve_graph()
        tr.train_batch(tuple(torch.from_numpy(r[:96].copy()) for r in rows))
        torch.cuda.synchronize()
    finally:
        ops.EncoderPassFn.forward, ops.EncoderPassFn.backward = staticmethod(f0), staticmethod(b0)
        losshead.LossHeadFn._backward_stage = staticmethod(h0)
    assert calls == {'fwd': 5, 'bwd': 5, 'head': 1}


class _Count:
    """Counts the calls made through an operator namespace (torch.ops.c2dsr / c2dsr_raw)."""

    def __init__(self, ns, tally, tag):
        self._ns, self._tally, self._tag = ns, tally, tag

    def __getattr__(self, name):
        op = getattr(self._ns, name)

        def call(*a, **k):
            self._tally[f'{self._tag}::{name}'] = self._tally.get(f'{self._tag}::{name}', 0) + 1
            return op(*a, **k)
        return call


def test_step_operator_calls():
    """a training step issues a few dozen operator calls (c2dsr:: stage operators plus the
    c2dsr_raw entry points still called one by one), not one call per kernel."""
    from c2dsr_amd import _lib
    rows, gs, gp = _case('fp32')
    args = make_args(C, dropout=0.2, precision='fp32', seed=5)
    args.batch_size = 96
    torch.manual_seed(1234)
    tr = build_trainer(args, gs, gp)
    tr.model.train()
    tr.optimizer.zero_grad()
    b = [tuple(torch.from_numpy(r[s * 96:(s + 1) * 96].copy()) for r in rows) for s in range(2)]
    tr.model.convolve_graph()
    tr.train_batch(b[0])  # warm-up: weight images made, plans cached
    torch.cuda.synchronize()
    tally = {}
    ops = _lib._load_ops()
    saved = dict(ops)
    ops['stage'], ops['raw'] = _Count(saved['stage'], tally, 'c2dsr'), _Count(saved['raw'], tally, 'c2dsr_raw')
    _lib.lib._fns.clear()
    try:
        tr.model.convolve_graph()
        tr.train_batch(b[1])
        torch.cuda.synchronize()
    finally:
        ops.update(saved)
        _lib.lib._fns.clear()
    raw = {k: v for k, v in tally.items() if k.startswith('c2dsr_raw::') and not k.endswith(('_workspace', '_bytes',
                                                                                               '_supported'))}
    n = sum(tally[k] for k in tally if k.startswith('c2dsr::')) + sum(raw.values())
    print('operator calls per step:', n, sorted(tally.items()))
    assert tally.get('c2dsr::encoder_pass') == 5 and tally.get('c2dsr::encoder_pass_backward') == 5
    assert n <= 48, (n, tally)
