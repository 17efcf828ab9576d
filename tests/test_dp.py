"""Data-parallel protocol on CPU (gloo, world_size 2): the product's row split (trainer.dp_rows), the
global-count loss normalisation and one sum all-reduce of the per-rank gradients reproduce the
single-device step exactly.  Per-rank compute is the oracle (CPU); the dropout masks
use the same global row offsets as the HIP kernels, so p > 0 is covered too."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from c2dsr_amd.trainer import dp_rows
from oracle import c2dsr_oracle as O
from tests import goldens as G


def test_dp_rows_split():
    for B in (16, 15, 1, 7):
        for world in (1, 2, 3, 4):
            got = [dp_rows(B, r, world) for r in range(world)]
            cover = [i for lo, hi, off, bg in got for i in range(lo, hi)]
            assert cover == list(range(B))
            assert all(off == lo and bg == B for lo, hi, off, bg in got)
    # weak scaling: own batch per rank, global row offsets disjoint
    assert [dp_rows(8, r, 4, dp_split=False)[2] for r in range(4)] == [0, 8, 16, 24]
    assert dp_rows(8, 1, 4, dp_split=False)[3] == 32


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg_name, p, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(1)
    cfg = G.oracle_cfg(cfg_name, p, p)
    batch = G.batch(cfg_name, 0, G.BATCH)
    lo, hi, off, _ = dp_rows(batch[0].shape[0], rank, world)
    local = tuple(x[lo:hi] for x in batch)
    counts = O.loss_counts(local, cfg)
    dist.all_reduce(counts)  # the 5 global counts (one tiny collective)
    tr = O.OracleTrainer(G.init_params(cfg_name), G.graphs_coo(cfg_name), cfg, seed=7)
    out = tr.train_batch(local, row_offset=off, optimizer=False, counts=counts)
    flat = torch.cat([tr.grads[n].reshape(-1) for n in tr.names if tr.grads[n] is not None])
    loss = torch.stack([out['loss'], out['loss_rec'], out['loss_mi']]).double()
    dist.all_reduce(flat)
    dist.all_reduce(loss)
    if rank == 0:
        np.save(os.path.join(out_dir, 'flat.npy'), flat.numpy())
        np.save(os.path.join(out_dir, 'loss.npy'), loss.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize('cfg_name,p', [('base', 0.0), ('var', 0.2)])
def test_dp_world2_equals_single_device(tmp_path, cfg_name, p):
    mp.spawn(_worker, args=(2, _free_port(), cfg_name, p, str(tmp_path)), nprocs=2, join=True)
    cfg = G.oracle_cfg(cfg_name, p, p)
    batch = G.batch(cfg_name, 0, G.BATCH)
    tr = O.OracleTrainer(G.init_params(cfg_name), G.graphs_coo(cfg_name), cfg, seed=7)
    out = tr.train_batch(batch, row_offset=0, optimizer=False)
    ref = torch.cat([tr.grads[n].reshape(-1) for n in tr.names if tr.grads[n] is not None]).numpy()
    got = np.load(tmp_path / 'flat.npy')
    loss = np.load(tmp_path / 'loss.npy')
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    np.testing.assert_allclose(loss, [float(out['loss']), float(out['loss_rec']), float(out['loss_mi'])], rtol=1e-5)


# ----------------------------------------------------------------------------- bucketed all-reduce (dp.py)
def _toy_store(shared):
    from c2dsr_amd.flat import FlatStore
    torch.manual_seed(0)
    e = torch.nn.Parameter(torch.randn(7, 5))
    ea = e if shared else torch.nn.Parameter(torch.randn(7, 5))
    eb = e if shared else torch.nn.Parameter(torch.randn(7, 5))
    pos = torch.nn.Parameter(torch.randn(3, 5))
    w = torch.nn.Parameter(torch.randn(6, 5))
    b = torch.nn.Parameter(torch.randn(6))
    named = [('embed_i.weight', e), ('embed_i_a.weight', ea), ('embed_i_b.weight', eb), ('pos', pos), ('w', w),
             ('b', b)]
    return FlatStore(named, torch.device('cpu')), (e, ea, eb)


class _Done:
    def wait(self):
        pass


@pytest.mark.parametrize('shared', [False, True])
def test_grad_buckets_cover_once(shared):
    from c2dsr_amd.dp import GradBuckets
    flat, tables = _toy_store(shared)
    seen = []
    gb = GradBuckets(flat, list(tables), n_lookups=5, allreduce=lambda t: seen.append(t) or _Done())
    for _ in range(4):
        gb.lookup_done()
    assert gb.issued == []
    gb.lookup_done()  # dense bucket final after the 5th lookup backward
    t_end = max(hi for _, hi in gb.table_range.values())
    assert len(gb.issued) >= 1 and all(lo >= t_end for lo, _ in gb.issued)
    for t in reversed(tables):  # GCN backwards run b, a, share
        gb.table_done(t)
    gb.finish()
    mark = torch.zeros(flat.numel, dtype=torch.int32)
    for lo, hi in gb.issued:
        mark[lo:hi] += 1
    for _, p, o, n in flat.entries:
        assert bool((mark[o:o + n] == 1).all())


def _bucket_worker(rank, world, port, out_dir):
    from c2dsr_amd.dp import GradBuckets
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    flat, tables = _toy_store(False)
    g = torch.Generator().manual_seed(100 + rank)
    flat.fresh.copy_(torch.randn(flat.numel, generator=g))
    full = flat.fresh.clone()
    dist.all_reduce(full)
    gb = GradBuckets(flat, list(tables), n_lookups=2)
    gb.lookup_done()
    gb.table_done(tables[2])  # a table may become final before the dense bucket
    gb.lookup_done()
    gb.table_done(tables[1])
    gb.table_done(tables[0])
    gb.finish()
    err = 0.0
    for _, p, o, n in flat.entries:
        err = max(err, float((flat.fresh[o:o + n] - full[o:o + n]).abs().max()))
    if rank == 0:
        np.save(os.path.join(out_dir, 'err.npy'), np.array([err]))
    dist.destroy_process_group()


def test_grad_buckets_world2_equal_full_allreduce(tmp_path):
    mp.spawn(_bucket_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert float(np.load(tmp_path / 'err.npy')[0]) == 0.0
