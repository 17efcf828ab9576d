"""End-to-end parity of the HIP training step with the reference (golden vectors,
dropout 0) and with the CPU oracle (dropout ON, identical hash masks).
Tolerance: 1e-4 relative (fp32 MFMA path), as north_star states."""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from tests import goldens as G

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL = 1e-4


def rel(a, b):
    a = np.asarray(a.detach().cpu() if isinstance(a, torch.Tensor) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if isinstance(b, torch.Tensor) else b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def make_args(c, dropout=0.0, precision='fp32', seed=0):
    n = c['n_a'] + c['n_b'] + 1
    return SimpleNamespace(d_latent=c['d_latent'], n_item=n, n_item_a=c['n_a'], n_item_b=c['n_b'], idx_pad=n - 1,
                           shared_item_embed=c['shared_item_embed'], d_bias=c['d_bias'], n_gnn=c['n_gnn'],
                           dropout_gnn=dropout, n_attn=c['n_attn'], n_head=c['n_head'], dropout_attn=dropout,
                           norm_first=c['norm_first'], len_max=c['len_max'], len_rec=c['len_rec'], lambda_loss=0.7,
                           lr=1e-3, l2=5e-4, lr_step=10, lr_gamma=0.5, batch_size=16, device=torch.device(DEV),
                           precision=precision, seed=seed)


def build_trainer(args, g_share, g_spec, params=None):
    from c2dsr_amd.trainer import Trainer
    tr = Trainer(args, None, data=(None, None, None), graphs=(g_share, g_spec))
    if params is not None:
        with torch.no_grad():
            for n, p in tr.model.named_parameters():
                if n in params:
                    p.copy_(params[n].to(DEV))
    return tr


def capture(tr):
    """Record the encoder outputs and hi tables of the next train_batch, and the grads before the step."""
    box = {}
    m = tr.model
    orig_fwd, orig_share, orig_step = m.forward, m.forward_share, tr.optimizer.step

    def fwd(*a):
        # rows of each encoder pass the loss reads (the last layer is computed only there in training)
        box['need'] = {pid: rs.idx[:rs.n].long().cpu() for pid, rs in m.state.need.items()}
        out = orig_fwd(*a)
        box['h_share'], box['hx'], box['hy'] = [o.detach().clone() for o in out]
        box['hi_share'], box['hi_a'], box['hi_b'] = m.hi_share.clone(), m.hi_a.clone(), m.hi_b.clone()
        return out

    def fsh(seq, pos):
        out = orig_share(seq, pos)
        box.setdefault('neg', []).append(out.detach().clone())
        return out

    def step():
        torch.cuda.synchronize()
        box['grads'] = {n: m.flat.grad_total(n).detach().cpu().clone() for n in m.flat.names}
        return orig_step()

    m.forward, m.forward_share, tr.optimizer.step = fwd, fsh, step
    return box


def read_rows(box, key, got, ref):
    """(got, ref) restricted to the rows the loss reads when the pass ran compacted, else whole."""
    from c2dsr_amd import dropout as DK
    pid = {'h_share': DK.PASS_SHARE, 'hx': DK.PASS_A, 'hy': DK.PASS_B, 'neg0': DK.PASS_NEG0,
           'neg1': DK.PASS_NEG0 + 1}.get(key)
    idx = box.get('need', {}).get(pid)
    ref = torch.as_tensor(np.asarray(ref))
    if idx is None:
        return got, ref
    d = got.shape[-1]
    if got.dim() == 2 and got.shape[0] == idx.numel():  # the pass's output holds just these rows
        return got.cpu(), ref.reshape(-1, d)[idx]
    return got.reshape(-1, d).cpu()[idx], ref.reshape(-1, d)[idx]


def golden_graphs(name):
    from c2dsr_amd.graph import CSRGraph
    g = G.load(f'graph_{name}.npz')
    n = int(g['n'])
    out = []
    for k in ('share', 'specific'):
        r, c, v = g[f'{k}_row'], g[f'{k}_col'], g[f'{k}_val']
        order = np.lexsort((c, r))
        r, c, v = r[order], c[order], v[order]
        rowptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
        out.append(CSRGraph(n, rowptr.astype(np.int32), c.astype(np.int32), v.astype(np.float32)))
    return out


@pytest.mark.parametrize('compact', [True, False], ids=['compact', 'full'])
@pytest.mark.parametrize('name', list(G.CONFIGS))
def test_train_steps_match_reference(name, compact):
    m = G.load(f'model_{name}.npz')
    c = G.CONFIGS[name]
    args = make_args(c)
    gs, gp = golden_graphs(name)
    tr = build_trainer(args, gs, gp, G.init_params(name))
    tr.compact_rows = compact
    tr.model.train()
    tr.optimizer.zero_grad()
    for s in range(int(m['n_steps'])):
        b = G.batch(name, int(m[f's{s}/batch_lo']), int(m[f's{s}/batch_n']))
        box = capture(tr)
        tr.model.convolve_graph()
        loss, loss_rec, loss_mi = tr.train_batch(b)
        torch.cuda.synchronize()
        for k in ('hi_share', 'hi_a', 'hi_b', 'h_share', 'hx', 'hy'):
            assert rel(*read_rows(box, k, box[k], m[f's{s}/{k}'])) < TOL, (s, k)
        assert rel(*read_rows(box, 'neg0', box['neg'][0], m[f's{s}/h_neg_a'])) < TOL
        assert rel(*read_rows(box, 'neg1', box['neg'][1], m[f's{s}/h_neg_b'])) < TOL
        if not compact:
            assert not box['need']
        for k, v in (('loss', loss), ('loss_rec', loss_rec), ('loss_mi', loss_mi)):
            assert abs(float(v) - float(m[f's{s}/{k}'])) <= TOL * abs(float(m[f's{s}/{k}'])), (s, k)
        for n, gv in box['grads'].items():
            assert rel(gv, m[f's{s}/grad/{n}']) < TOL, (s, n)
        # continue from the reference's post-step parameters (AdamW turns rounding noise in
        # ~zero gradients into ±lr sign noise; the optimizer itself is checked separately)
        with torch.no_grad():
            for n, p in tr.model.named_parameters():
                key = f's{s}/param/{n}'
                if key in m.files:
                    ref = torch.from_numpy(m[key])
                    g = box['grads'].get(n)
                    if g is not None:
                        sig = g.abs() > 1e-3 * g.abs().max()
                        got = p.detach().cpu()
                        assert rel(got[sig], ref[sig]) < TOL, (s, n)
                        assert float((got - ref).abs().max()) <= 2.5e-3
                    p.copy_(ref.to(DEV))


@pytest.mark.parametrize('norm_first,n_head,n_gnn,n_attn', [(False, 1, 1, 1), (True, 2, 2, 1), (False, 2, 1, 2)])
def test_train_step_with_dropout_matches_oracle(norm_first, n_head, n_gnn, n_attn):
    """Larger synthetic case, dropout 0.2 everywhere: HIP step vs oracle with the same hash masks."""
    from c2dsr_amd import dataloader as DL
    from c2dsr_amd import graph as GR
    from c2dsr_amd import synth
    from oracle import c2dsr_oracle as O
    import random
    c = dict(n_a=300, n_b=400, len_max=20, len_rec=5, d_latent=64, n_gnn=n_gnn, n_attn=n_attn, n_head=n_head,
             norm_first=norm_first, d_bias=True, shared_item_embed=False)
    seqs = synth.make_sequences(200, c['n_a'], c['n_b'], c['len_max'], seed=3, n_min=4)
    random.seed(3407)
    rows = DL.to_arrays(DL.preprocess_train(seqs, c['n_a'], c['n_b'], c['len_max']))
    gs, gp = GR.preprocess_graph(seqs, c['n_a'], c['n_a'] + c['n_b'] + 1)
    args = make_args(c, dropout=0.2, seed=77)
    torch.manual_seed(0)
    tr = build_trainer(args, gs, gp)
    params = {n: p.detach().cpu().clone() for n, p in tr.model.named_parameters()}
    graphs = {}
    for k, g in (('share', gs), ('specific', gp)):
        r, cc, v = g.coo()
        graphs[k] = (torch.from_numpy(r), torch.from_numpy(cc), torch.from_numpy(v))
    ocfg = dict(d_latent=64, n_item_a=c['n_a'], n_item_b=c['n_b'], idx_pad=c['n_a'] + c['n_b'], len_rec=5,
                lambda_loss=0.7, n_gnn=n_gnn, n_attn=n_attn, n_head=n_head, norm_first=norm_first, d_bias=True,
                shared_item_embed=False, dropout_gnn=0.2, dropout_attn=0.2)
    orc = O.OracleTrainer(params, graphs, ocfg, seed=77)
    orc.step_no = 1  # the model's first convolve_graph opens step 1
    tr.model.train()
    tr.optimizer.zero_grad()
    B = 48
    for s in range(2):
        b = tuple(torch.from_numpy(r[s * B:(s + 1) * B].copy()) for r in rows)
        box = capture(tr)
        tr.model.convolve_graph()
        loss, loss_rec, loss_mi = tr.train_batch(b)
        out = orc.train_batch(b, optimizer=False)
        for k in ('hi_share', 'h_share', 'hx', 'hy'):
            assert rel(*read_rows(box, k, box[k], out[k])) < TOL, (s, k)
        assert abs(float(loss) - float(out['loss'])) < TOL * abs(float(out['loss']))
        for n in orc.names:
            assert rel(box['grads'][n], orc.grads[n]) < 5 * TOL, (s, n)
        with torch.no_grad():
            orc.opt.step(orc.P, orc.grads)
        for n, p in tr.model.named_parameters():
            if n in orc.names:
                g = orc.grads[n]
                sig = g.abs() > 1e-3 * g.abs().max()
                assert rel(p.detach().cpu()[sig], orc.P[n][sig]) < TOL, (s, n)
        with torch.no_grad():  # re-sync (sign noise of ~zero grads)
            for n, p in tr.model.named_parameters():
                if n in orc.names:
                    p.copy_(orc.P[n].to(DEV))
        orc.step_no = tr.model.state.step + 1


def test_bf16_step_close_to_fp32():
    """bf16-MFMA performance mode stays close to the fp32 parity mode (documented tolerance 2e-2)."""
    name = 'base'
    m = G.load(f'model_{name}.npz')
    c = G.CONFIGS[name]
    gs, gp = golden_graphs(name)
    tr = build_trainer(make_args(c, precision='bf16'), gs, gp, G.init_params(name))
    tr.model.train()
    tr.optimizer.zero_grad()
    b = G.batch(name, 0, 16)
    tr.model.convolve_graph()
    loss, _, _ = tr.train_batch(b)
    assert abs(float(loss) - float(m['s0/loss'])) < 2e-2 * abs(float(m['s0/loss']))
    assert math.isfinite(float(loss))


def _dp_gpu_worker(rank, world, port, name, out_dir):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        gs, gp = golden_graphs(name)
        tr = build_trainer(make_args(G.CONFIGS[name]), gs, gp, G.init_params(name))
        assert tr.world == world and tr.dp_split
        tr.model.train()
        tr.optimizer.zero_grad()
        box = capture(tr)
        tr.model.convolve_graph()
        loss, _, _ = tr.train_batch(G.batch(name, 0, G.BATCH))
        torch.cuda.synchronize()
        if rank == 0:
            np.savez(os.path.join(out_dir, 'dp.npz'), loss=float(loss), **{f'g/{n}': v.numpy()
                                                                           for n, v in box['grads'].items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('name', ['base', 'shared'])
def test_dp_world2_bucketed_allreduce_matches_reference(tmp_path, name):
    """Two data-parallel ranks on cuda:0 (gloo carries the collectives here; RCCL on the 8-GPU node):
    the row split + global-count normalisation + bucketed all-reduce issued inside the backward
    (c2dsr_amd/dp.py) reproduce the reference's single-device gradient."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    mp.spawn(_dp_gpu_worker, args=(2, port, name, str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / 'dp.npz')
    m = G.load(f'model_{name}.npz')
    assert abs(float(got['loss']) - float(m['s0/loss'])) <= TOL * abs(float(m['s0/loss']))
    names = [k[2:] for k in got.files if k.startswith('g/')]
    assert names
    for n in names:
        assert rel(got[f'g/{n}'], m[f's0/grad/{n}']) < TOL, n
