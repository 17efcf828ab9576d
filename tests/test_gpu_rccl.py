"""RCCL itself on the one-GPU box (missing #1).

The 8-GPU node is the driver's; every earlier GPU test ran the data-parallel exchange through gloo (two ranks on one
device, which RCCL refuses).  A process group of ONE rank is something RCCL accepts, and with C2DSR_DP_FORCE=1 the
trainer runs the full data-parallel step on it — so every RCCL call of the exchange executes on the real library:
  * init_data_parallel's 'nccl' + device_id branch (trainer.py), from the launcher's environment only;
  * DPComm's async all-reduce per reduction range (dp.py: dist.all_reduce(..., async_op=True));
  * ZeRO-1's reduce_scatter_tensor / all_gather_into_tensor (dp.py reduce_scatter / all_gather, not their gloo
    fallbacks);
  * RowShard's all-gathers of the propagated tables (ops.RowShard, C2DSR_GNN_SHARD=1; var: n_gnn = 2, so an
    intermediate round's synchronous gather too).
A one-rank sum is the identity, and from a zero accumulator the data-parallel step's fresh-gradient fold adds
exactly zero, so the step must be BIT-equal to the non-DP step (trainer.py:156-158 reference semantics)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests import goldens as G
from tests.test_gpu_parity import build_trainer, golden_graphs, make_args

pytestmark = pytest.mark.gpu

MODES = {'allreduce': {}, 'zero1': {'C2DSR_ZERO1': '1'}, 'gnn_shard': {'C2DSR_GNN_SHARD': '1'},
         'zero1_gnn_shard': {'C2DSR_ZERO1': '1', 'C2DSR_GNN_SHARD': '1'}}


def _one_step(name):
    gs, gp = golden_graphs(name)
    tr = build_trainer(make_args(G.CONFIGS[name], dropout=0.2), gs, gp, G.init_params(name))
    tr.model.train()
    tr.optimizer.zero_grad()
    tr.model.convolve_graph()
    loss, loss_rec, loss_mi = tr.train_batch(G.batch(name, 0, 16))
    torch.cuda.synchronize()
    return tr, np.array([float(loss.detach()), float(loss_rec), float(loss_mi)])


def _rank(rank, port, name, mode, out_dir):
    os.environ.update(RANK='0', LOCAL_RANK='0', WORLD_SIZE='1', LOCAL_WORLD_SIZE='1', MASTER_ADDR='127.0.0.1',
                      MASTER_PORT=str(port), C2DSR_DP_FORCE='1', C2DSR_ZERO1='0', C2DSR_GNN_SHARD='0')
    os.environ.update(MODES[mode])
    import torch.distributed as dist
    from c2dsr_amd import dp
    calls = {'all_reduce': 0, 'reduce_scatter_tensor': 0, 'all_gather_into_tensor': 0}
    for fn in calls:  # count the RCCL entry points the step reaches (the gloo fallbacks never call these)
        orig = getattr(dist, fn)

        def wrap(*a, _o=orig, _n=fn, **k):
            calls[_n] += 1
            return _o(*a, **k)
        setattr(dist, fn, wrap)
    try:
        tr, losses = _one_step(name)  # Trainer(...) initialises the group itself (init_data_parallel)
        assert dist.is_initialized() and dist.get_backend() == 'nccl', dist.get_backend()
        assert tr.dp and tr.world == 1 and not tr.model.flat.direct
        assert not dp._gloo_cuda(tr.model.flat.fresh)
        assert (tr.zero is not None) == ('zero1' in mode)
        assert (tr.model.row_shard is not None) == ('gnn_shard' in mode)
        np.savez(os.path.join(out_dir, f'{mode}.npz'), losses=losses,
                 calls=np.array([calls[k] for k in sorted(calls)]),
                 **{f'p/{n}': p.detach().cpu().numpy() for n, p in tr.model.named_parameters()})
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('name', ['base', 'var'])
def test_rccl_world1_dp_step_is_bit_equal_to_the_single_device_step(tmp_path, name):
    for mode in MODES:  # one spawned process per mode (a fresh RCCL group each), one after another
        mp.spawn(_rank, args=(_free_port(), name, mode, str(tmp_path)), nprocs=1, join=True)
    tr, losses = _one_step(name)
    assert not tr.dp
    want = {n: p.detach().cpu().numpy() for n, p in tr.model.named_parameters()}
    for mode in MODES:
        got = np.load(tmp_path / f'{mode}.npz')
        n_gather, n_allreduce, n_rs = (int(v) for v in got['calls'])  # sorted names
        assert n_allreduce > 0, mode  # the valid-target counts ahead of the forward, at least
        if 'zero1' in mode:
            assert n_rs > 0 and n_gather > 0, (mode, n_rs, n_gather)
        if 'gnn_shard' in mode:
            assert n_gather > 0, mode
        if 'zero1' not in mode:
            assert n_allreduce > 1, mode  # the gradient ranges too
        np.testing.assert_array_equal(got['losses'], losses, err_msg=mode)
        for n, w in want.items():
            np.testing.assert_array_equal(got[f'p/{n}'], w, err_msg=f'{mode}: {n}')
