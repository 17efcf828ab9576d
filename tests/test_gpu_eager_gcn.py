"""A table's GCN backward runs as soon as the last lookup of its propagated table has run its backward
(ops.GradSink.lookup_done), not where autograd schedules GCNFn's node (after every other node): data-parallel
steps then issue each item table's collectives under the remaining passes' backward (dp.py).  Same kernels on
the same inputs, so the step is bit-identical to the autograd-ordered one."""
import pytest
import torch

from c2dsr_amd import ops
from tests import goldens as G
from tests.test_gpu_parity import build_trainer, golden_graphs, make_args

pytestmark = pytest.mark.gpu


def _run(eager, name, steps=2):
    ops.EAGER_GCN = eager
    try:
        gs, gp = golden_graphs(name)
        tr = build_trainer(make_args(G.CONFIGS[name]), gs, gp, G.init_params(name))
        tr.model.train()
        tr.optimizer.zero_grad()
        events = []
        gb, nl = ops.gcn_backward, ops.notify_lookup

        def gcn_rec(sink, *a):
            events.append('gcn')
            return gb(sink, *a)

        def look_rec(state):
            events.append('lookup')
            return nl(state)
        ops.gcn_backward, ops.notify_lookup = gcn_rec, look_rec
        try:
            losses = []
            for s in range(steps):
                b = G.batch(name, 16 * s, 16)
                tr.model.convolve_graph()
                loss, _, _ = tr.train_batch(b)
                losses.append(loss.detach().clone())
        finally:
            ops.gcn_backward, ops.notify_lookup = gb, nl
        torch.cuda.synchronize()
        return tr.model.flat.param.clone(), tr.model.flat.accum.clone(), losses, events
    finally:
        ops.EAGER_GCN = True


@pytest.mark.parametrize('name', ['base', 'var', 'shared'])
def test_eager_gcn_backward_is_bit_identical_and_early(name):
    p1, a1, l1, ev1 = _run(True, name)
    p0, a0, l0, ev0 = _run(False, name)
    assert torch.equal(p1, p0) and torch.equal(a1, a0), 'eager GCN backward changed the step'
    assert all(torch.equal(x, y) for x, y in zip(l1, l0))
    step = ev1[:len(ev1) // 2]
    # five lookups and three table backwards per step; eagerly, two tables' backwards run before the last lookup
    assert step.count('lookup') == 5 and step.count('gcn') == 3, step
    last = max(i for i, e in enumerate(step) if e == 'lookup')
    assert sum(1 for e in step[:last] if e == 'gcn') == 2, step
    assert ev0[:len(ev0) // 2] == ['lookup'] * 5 + ['gcn'] * 3  # autograd's order: every table at the end
