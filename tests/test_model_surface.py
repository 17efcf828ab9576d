"""CPU checks of the drop-in module surface: parameter names, shapes and the
initialisation (same torch RNG draws as the reference, so equal state_dicts for
the same seed), the C-ABI library exports, and the header-derived binding."""
import torch

from tests import goldens as G
from tests.test_gpu_parity import golden_graphs, make_args


def test_init_matches_reference_state_dict():
    from c2dsr_amd.models.C2DSR import C2DSR
    for name in G.CONFIGS:
        args = make_args(G.CONFIGS[name])
        args.device = torch.device('cpu')
        gs, gp = golden_graphs(name)
        torch.manual_seed(1234)  # tools/gen_fixtures.py seeds the reference model with 1234
        model = C2DSR(args, gs, gp)
        ref = G.init_params(name)
        sd = model.state_dict()
        assert set(ref) <= set(sd), set(ref) - set(sd)
        for k, v in ref.items():
            assert torch.equal(sd[k], v), (name, k)


def test_library_exports_every_declared_symbol():
    import ctypes
    from c2dsr_amd._lib import LIB_PATH, parse_header
    lib = ctypes.CDLL(LIB_PATH)
    sigs = parse_header()
    assert len(sigs) >= 25
    for name in sigs:
        assert hasattr(lib, name), name


def test_trainable_parameters_exclude_template_layer():
    from c2dsr_amd.models.C2DSR import C2DSR
    args = make_args(G.CONFIGS['base'])
    args.device = torch.device('cpu')
    gs, gp = golden_graphs('base')
    model = C2DSR(args, gs, gp)
    names = [n for n, _ in model.trainable_named_parameters()]
    assert not any('.encoder_layer.' in n for n in names)
    m = G.load('model_base.npz')
    assert set(names) == {k[len('s0/grad/'):] for k in m.files if k.startswith('s0/grad/')}


def test_convolve_graph_defers_the_propagation_to_first_use():
    """C2DSR.convolve_graph (C2DSR.py:59-62) opens the dropout step at once but enqueues the three GCN propagations at
    the first read of a table — hi_* / forward, or earlier by the trainer right after its index work — under the
    grad / train modes of the convolve_graph call, once per call."""
    from c2dsr_amd.models.C2DSR import C2DSR
    args = make_args(G.CONFIGS['base'])
    args.device = torch.device('cpu')
    gs, gp = golden_graphs('base')
    model = C2DSR(args, gs, gp)
    calls = []

    def stub(gnn):
        def propagate(h, adj, sink=None, shard=None):
            calls.append((gnn.table, gnn.training, torch.is_grad_enabled()))
            return h * (gnn.table + 1), None, None
        return propagate

    for g in (model.gnn_share, model.gnn_a, model.gnn_b):
        g.propagate = stub(g)
    model.defer_graph = True  # as c2dsr_amd.Trainer sets it
    model.train()
    step0 = model.state.step
    model.convolve_graph()
    assert model.state.step == step0 + 1 and calls == []  # nothing enqueued yet
    model.eval()  # a mode change after the call does not change the propagation's mode
    with torch.no_grad():
        hs = model.hi_share
    assert calls == [(0, True, True), (1, True, True), (2, True, True)]
    assert torch.equal(hs, model.embed_i.weight)
    assert torch.equal(model.hi_b, model.embed_i_b.weight * 3)
    assert len(calls) == 3  # launched once per convolve_graph
    with torch.no_grad():
        model.convolve_graph()
    model.launch_graph()
    assert calls[3:] == [(0, False, False), (1, False, False), (2, False, False)]
    assert model.state.step == step0 + 1  # eval calls open no dropout step


def test_convolve_graph_is_eager_unless_trainer_driven_and_guards_weight_edits():
    """a model used on its own propagates at convolve_graph() like the reference; a deferred
    (trainer-driven) launch refuses item-embedding weights edited in place between the call and the first read."""
    import pytest
    from c2dsr_amd.models.C2DSR import C2DSR
    args = make_args(G.CONFIGS['base'])
    args.device = torch.device('cpu')
    gs, gp = golden_graphs('base')
    model = C2DSR(args, gs, gp)
    calls = []
    for g in (model.gnn_share, model.gnn_a, model.gnn_b):
        g.propagate = (lambda gnn: lambda h, adj, sink=None, shard=None: (calls.append(gnn.table), (h.clone(), None,
                                                                                                   None))[1])(g)
    model.train()
    model.convolve_graph()
    assert calls == [0, 1, 2]  # eager
    assert torch.equal(model.hi_a, model.embed_i_a.weight)
    model.defer_graph = True
    model.convolve_graph()
    assert calls == [0, 1, 2]
    with torch.no_grad():
        model.embed_i_a.weight.add_(1.0)  # e.g. an optimizer step between the call and the first read
    with pytest.raises(RuntimeError, match='modified between convolve_graph'):
        model.hi_a
    model.convolve_graph()  # a new call sees the new weights
    assert torch.equal(model.hi_a, model.embed_i_a.weight) and calls == [0, 1, 2, 0, 1, 2]
    # the fused optimizer writes the weights through a kernel (no _version bump) and bumps
    # ops.WEIGHTS.epoch instead — a step between the call and the first read is refused as well
    from c2dsr_amd import ops
    model.convolve_graph()
    ops.WEIGHTS.epoch += 1  # what FlatAdamW.step() → WEIGHTS.bump() does after its kernel
    with pytest.raises(RuntimeError, match='modified between convolve_graph'):
        model.hi_b
    model.convolve_graph()
    assert torch.equal(model.hi_b, model.embed_i_b.weight)
