"""Data parallelism under the reference's UNCHANGED main.py.

A scratch checkout is assembled the way INTEGRATION.md §2 says — the reference's own main.py and utils/ with
the dropin/ shims copied over trainer.py, dataloader.py, models/ and utils/graph.py — and main.py is launched
by torchrun with two processes on the host (`--cuda cpu`).  The drop-in Trainer must set up the process group
itself (c2dsr_amd.trainer.init_data_parallel: gloo here, RCCL on a GPU node), give every rank its own device,
and then stop at the first kernel with HipLibError, since there is no CPU fallback.  The two-rank run on the
GPU is tests/test_gpu_dropin_dp.py.

The reference is read from /root/reference at test time (this container only); the test is skipped where it
is absent (the GPU box)."""
import hashlib
import os
import shutil
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = '/root/reference'


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def checkout(dst):
    """The reference checkout with the dropin/ files copied over it."""
    for sub in ('', 'models', 'utils'):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
        src = os.path.join(REF, sub)
        for f in os.listdir(src):
            if f.endswith('.py'):
                shutil.copy(os.path.join(src, f), os.path.join(dst, sub, f))
    for rel in ('trainer.py', 'dataloader.py', 'models/C2DSR.py', 'models/encoders.py', 'utils/graph.py'):
        shutil.copy(os.path.join(ROOT, 'dropin', rel), os.path.join(dst, rel))
    # main.py's default (processed) input path: data/Food-Kitchen/{train,val,test}.pkl + graph.pkl + items_*.txt
    shutil.copytree(os.path.join(ROOT, 'tests', 'golden', 'processed_base'), os.path.join(dst, 'data', 'Food-Kitchen'))
    return dst


def _sha(p):
    return hashlib.sha256(open(p, 'rb').read()).hexdigest()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, 'main.py')), reason='reference checkout absent')
def test_torchrun_unchanged_main_sets_up_data_parallel(tmp_path):
    co = checkout(str(tmp_path / 'co'))
    assert _sha(os.path.join(co, 'main.py')) == _sha(os.path.join(REF, 'main.py'))  # byte-for-byte
    env = dict(os.environ, C2DSR_AMD_ROOT=ROOT, PYTHONDONTWRITEBYTECODE='1', OMP_NUM_THREADS='1')
    env.pop('WORLD_SIZE', None)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(_free_port()), 'main.py', '--cuda', 'cpu', '--d_latent', '32',
           '--batch_size', '16', '--n_epoch', '1', '--num_workers', '0']
    r = subprocess.run(cmd, cwd=co, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    # every rank got its own process group membership from the launcher's environment, on its device
    assert '[c2dsr] data parallel: rank 0/2 on cpu (gloo)' in out, out[-3000:]
    assert '[c2dsr] data parallel: rank 1/2 on cpu (gloo)' in out, out[-3000:]
    # both ranks reached the training loop (main.py:113) and stopped at the first kernel: no CPU fallback
    assert out.count('[Epoch 1]') == 2, out[-3000:]
    assert 'HipLibError' in out and 'no CPU fallback' in out, out[-3000:]
    assert r.returncode != 0


def test_init_data_parallel_outside_a_launcher_is_a_no_op(monkeypatch):
    from types import SimpleNamespace
    import torch
    from c2dsr_amd.trainer import init_data_parallel
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    args = SimpleNamespace(device=torch.device('cuda:3'))
    assert init_data_parallel(args) == (0, 1)
    assert args.device == torch.device('cuda:3')  # main.py's single-process device is kept


def test_dp_backend_from_device_identities():
    """the backend follows the ranks' physical devices, not the local device count — a launcher
    that gives every rank its own HIP_VISIBLE_DEVICES leaves each rank one visible device, yet each drives its own
    GPU (RCCL); only ranks that really share a GPU fall back to gloo, and every rank reaches the same answer."""
    from c2dsr_amd.trainer import dp_backend
    own = [f'node0|0:{b}:0|uuid{b}' for b in (3, 4, 5, 6)]
    assert all(dp_backend(own, r) == 'nccl' for r in range(4))
    shared = ['node0|0:3:0|u', 'node0|0:3:0|u']
    assert all(dp_backend(shared, r) == 'gloo' for r in range(2))
    mixed = ['node0|0:3:0|u', 'node0|0:3:0|u', 'node0|0:4:0|v']
    assert {dp_backend(mixed, r) for r in range(3)} == {'gloo'}
    # the same bus number on two hosts is two GPUs
    assert dp_backend(['a|0:3:0|u', 'b|0:3:0|u'], 0) == 'nccl'
