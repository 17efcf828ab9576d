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


# ----------------------------------------------------------------------------- gradient exchange (dp.py)
def _toy_store(shared, world=2, N=37, d=8, with_head=False):
    from c2dsr_amd.flat import FlatStore
    torch.manual_seed(0)
    e = torch.nn.Parameter(torch.randn(N, d))
    ea = e if shared else torch.nn.Parameter(torch.randn(N, d))
    eb = e if shared else torch.nn.Parameter(torch.randn(N, d))
    pos = torch.nn.Parameter(torch.randn(3, d))
    w = torch.nn.Parameter(torch.randn(6, d))
    b = torch.nn.Parameter(torch.randn(6))
    ca = torch.nn.Parameter(torch.randn(11, d))
    cb = torch.nn.Parameter(torch.randn(11))
    named = [('pos', pos), ('embed_i.weight', e), ('embed_i_a.weight', ea), ('w', w), ('embed_i_b.weight', eb),
             ('b', b), ('classifier_a.weight', ca), ('classifier_a.bias', cb)]
    st = FlatStore(named, torch.device('cpu'), align=4 * world)
    return (st, (e, ea, eb), (ca, cb)) if with_head else (st, (e, ea, eb))


class _Done:
    def wait(self):
        pass


@pytest.mark.parametrize('world', [1, 2, 3, 4, 8])
@pytest.mark.parametrize('shared', [False, True])
def test_comm_plan_tiles_flat_store(world, shared):
    from c2dsr_amd.dp import CommPlan, Zero1
    flat, tables = _toy_store(shared, world)
    plan = CommPlan(flat, list(tables), world)
    mark = torch.zeros(flat.numel, dtype=torch.int32)
    for lo, hi in plan.ranges:
        assert (hi - lo) % (4 * world) == 0 and lo % 4 == 0
        mark[lo:hi] += 1
    assert bool((mark == 1).all())
    for ch in plan.table_chunks.values():  # row chunks are consecutive and cover the table
        assert ch[0][0] == 0 and all(a[1] == b[0] for a, b in zip(ch, ch[1:]))
    own = torch.zeros(flat.numel, dtype=torch.int32)
    for r in range(world):  # the ranks' ZeRO-1 parts partition every range
        z = Zero1(flat, plan, r, world, gather=lambda o, i: _Done())
        for lo, hi, olo, ohi, off in z.parts:
            assert lo <= olo < ohi <= hi and (ohi - olo) * world == hi - lo
            own[olo:ohi] += 1
        assert z.shard_numel * world == flat.numel
    assert bool((own == 1).all())


def test_head_ranges_issue_first():
    """The classifier / discriminator range goes out when the loss head's backward returns, before the
    encoder (dense) ranges and the tables; all ranges still tile the store exactly once."""
    from c2dsr_amd.dp import CommPlan, DPComm
    flat, tables, head = _toy_store(False, with_head=True)
    plan = CommPlan(flat, list(tables), 2, head=list(head))
    assert len(plan.head) == 1  # contiguous slices merged
    dc = DPComm(flat, plan, 1, list(tables), reduce=lambda lo, hi: _Done())
    dc.head_done()
    assert dc.issued == plan.head
    dc.lookup_done()
    assert dc.issued == plan.head + plan.dense
    for t in tables:
        dc.table_done(t)
    dc.finish()
    assert sorted(dc.issued) == sorted(plan.ranges)


@pytest.mark.parametrize('shared', [False, True])
def test_dpcomm_issue_points(shared):
    """Dense ranges after the last lookup backward; a table's chunks as its last GCN backward writes
    them (earlier GCN backwards of a shared table issue nothing); finish() covers the rest once."""
    from c2dsr_amd.dp import CommPlan, DPComm
    flat, tables = _toy_store(shared)
    plan = CommPlan(flat, list(tables), 2)
    seen = []
    dc = DPComm(flat, plan, 5, list(tables), reduce=lambda lo, hi: seen.append((lo, hi)) or _Done())
    for _ in range(4):
        dc.lookup_done()
    assert dc.issued == []
    dc.lookup_done()
    assert dc.issued == plan.dense
    for k, t in enumerate(reversed(tables)):  # GCN backwards run b, a, share
        cuts = dc.row_cuts(t)
        last = not shared or k == 2
        assert (cuts is not None) == last
        n0 = len(dc.issued)
        if cuts:
            for r0, r1 in cuts:
                dc.table_rows_done(t, r0, r1)
                assert len(dc.issued) > n0
                n0 = len(dc.issued)
        dc.table_done(t)
    dc.finish()
    assert sorted(dc.issued) == sorted(plan.ranges) and len(seen) == len(plan.ranges)


def _zero_worker(rank, world, port, shared, out_dir):
    """Two AdamW steps with epoch accumulation: replicated (all-reduce + update of everything) vs ZeRO-1
    (reduce-scatter per range + update of the owned parts + all-gather).  Gradients are small integers so
    every summation order is exact: the parameters must be bit-equal on every rank."""
    from c2dsr_amd.dp import CommPlan, DPComm, Zero1
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.set_num_threads(1)
    flat, tables = _toy_store(shared, world)
    plan = CommPlan(flat, list(tables), world)
    zero = Zero1(flat, plan, rank, world)
    ref_p = flat.param.clone()
    ref_acc = torch.zeros(flat.numel)
    ref_opt, z_opt = O.AdamWAmsgrad(), O.AdamWAmsgrad()
    z_acc = torch.zeros(zero.shard_numel)
    g = torch.Generator().manual_seed(100 + rank)
    for step in range(2):
        fresh = torch.randint(-8, 9, (flat.numel,), generator=g).float()
        full = fresh.clone()
        dist.all_reduce(full)
        ref_acc += full
        ref_opt.step({'all': ref_p}, {'all': ref_acc.clone()})
        flat.fresh.copy_(fresh)
        dc = DPComm(flat, plan, 1, list(tables), zero=zero)
        for t in reversed(tables):
            for r0, r1 in dc.row_cuts(t) or []:
                dc.table_rows_done(t, r0, r1)
            dc.table_done(t)
        dc.lookup_done()
        dc.finish()
        for k, (lo, hi, olo, ohi, off) in enumerate(zero.parts):
            sl = slice(off, off + ohi - olo)
            assert torch.equal(zero.gshard[sl], full[olo:ohi])
            z_acc[sl] += zero.gshard[sl]
            z_opt.step({k: flat.param[olo:ohi]}, {k: z_acc[sl].clone()})
        for w in zero.gather():
            w.wait()
        if not torch.equal(flat.param, ref_p):
            raise AssertionError(f'rank {rank} step {step}: ZeRO-1 params differ by '
                                 f'{float((flat.param - ref_p).abs().max())}')
    if rank == 0:
        np.save(os.path.join(out_dir, 'ok.npy'), np.array([1]))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,shared', [(2, False), (4, False), (4, True)])
def test_zero1_equals_replicated_allreduce(tmp_path, world, shared):
    mp.spawn(_zero_worker, args=(world, _free_port(), shared, str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / 'ok.npy').exists()


def _bucket_worker(rank, world, port, out_dir):
    from c2dsr_amd.dp import CommPlan, DPComm
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    flat, tables = _toy_store(False, world)
    g = torch.Generator().manual_seed(100 + rank)
    flat.fresh.copy_(torch.randn(flat.numel, generator=g))
    full = flat.fresh.clone()
    dist.all_reduce(full)
    dc = DPComm(flat, CommPlan(flat, list(tables), world), 2, list(tables))
    dc.lookup_done()
    dc.table_done(tables[2])  # a table may become final before the dense ranges
    dc.lookup_done()
    for r0, r1 in dc.row_cuts(tables[1]):
        dc.table_rows_done(tables[1], r0, r1)
    dc.table_done(tables[1])
    dc.table_done(tables[0])
    dc.finish()
    err = float((flat.fresh - full).abs().max())
    if rank == 0:
        np.save(os.path.join(out_dir, 'err.npy'), np.array([err]))
    dist.destroy_process_group()


def test_allreduce_ranges_world2_equal_full_allreduce(tmp_path):
    mp.spawn(_bucket_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert float(np.load(tmp_path / 'err.npy')[0]) == 0.0


@pytest.mark.parametrize('world', [2, 3, 8])
@pytest.mark.parametrize('n', [1, 7, 101, 100783])
def test_row_shard_blocks_tile_the_table(world, n):
    """ops.RowShard (row-sharded GCN propagation): the ranks' row blocks tile [0, n) in rank
    order, every block (but a tail one) has ⌈n/world⌉ rows, and the padded buffer splits into world equal parts."""
    from c2dsr_amd.ops import RowShard
    pos = 0
    for r in range(world):
        sh = RowShard(r, world, gather=lambda out, inp: _Done())
        r0, r1 = sh.rows(n)
        assert r0 == pos and r1 >= r0
        assert r1 - r0 == sh.block(n) or r1 == n
        pos = r1
        buf = sh.buffer(torch.empty(n, 4))
        assert buf.shape == (sh.block(n) * world, 4) and buf.shape[0] >= n
    assert pos == n


def _shard_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from c2dsr_amd.ops import RowShard
        sh = RowShard(rank, world)
        n, d = 37, 8
        full = sh.buffer(torch.empty(n, d))
        full.fill_(-1.0)
        r0, r1 = sh.rows(n)
        ref = torch.arange(n * d, dtype=torch.float32).view(n, d)
        full[r0:r1] = ref[r0:r1]  # this rank's block only
        sh.pending.append(sh.gather(full))
        sh.wait()
        torch.save(full[:n].clone(), os.path.join(out_dir, f'g{rank}.pt'))
    finally:
        dist.destroy_process_group()


def test_row_shard_gather_world3(tmp_path):
    """The blocks written by each rank are all-gathered in place into every rank's full table (gloo, 3 ranks)."""
    port = _free_port()
    mp.spawn(_shard_worker, args=(3, port, str(tmp_path)), nprocs=3, join=True)
    ref = torch.arange(37 * 8, dtype=torch.float32).view(37, 8)
    for r in range(3):
        assert torch.equal(torch.load(tmp_path / f'g{r}.pt', weights_only=True), ref)
