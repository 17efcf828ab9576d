"""north_star: "Recall/MRR/NDCG@{5,20} reproduce on Food-Kitchen" (VERDICT r02 #6).

main.py's loop (main.py:88-148: seeding, Trainer(args, noter), run_epoch, the StepLR step, run_test,
cal_score) through the drop-in Trainer on the GPU, on the Food-Kitchen files the reference ships
(tests/golden/fk_raw.npz: data/raw/Food-Kitchen/{val.txt, test_new.txt, items_a.txt, items_b.txt}; the
train file is a missing blob, so train := val.txt, val := test := test_new.txt), at BASELINE configs[0]
(C1: d=64, L=15, B=128, R=10, 999 sampled negatives), dropout 0, fp32 mode — against the reference's own
run of the same loop (tests/golden/traj_fk.npz, tools/gen_fixtures.py --fk-traj).

Tolerances (stated): the shuffled batch order and the data construction are exact; the per-epoch losses
and every step loss of the first epoch within 1e-4 relative (north_star); the step losses of later epochs
within 1e-3 (the two trajectories drift apart through 60+ AdamW steps on rounding-level gradient
differences — measured 1.2e-4 on one of 180 values in epoch 2); ranks over 999 sampled negatives compare two
scores, so a near-tie can resolve differently under fp32 rounding (and, after the first epoch, under the
trajectories' drift) — at least 99.5 % of the ranks identical in the first epoch and 98.5 % later, 99.9 %
within ±1, and HR/MRR/NDCG@{5,20} of each domain (utils/metrics.py:4-19) within 1e-3 absolute.  Measured on
MI355X (round 4): first epoch 99.58-99.75 % identical ranks (val_a 99.75, val_b 99.61, test_a 99.64, test_b
99.58), 100 % within ±1, metrics within 8.8e-6; second epoch 98.99-99.31 % identical (val_a 99.27, val_b 98.99,
test_a 99.31, test_b 99.15), ≥ 99.96 % within ±1, metrics within 3.6e-4 — the thresholds leave 0.08 / 0.49 points of
headroom on identical ranks."""
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from tests import goldens as G

pytestmark = pytest.mark.gpu
BENCH_FK = [0.1124, 0.0865, 0.0574, 0.0416]  # utils/constant.py:14


class Noter:
    def __init__(self):
        self.train = []

    def log_train(self, *a):
        self.train.append(a[:3])


def _raw_dir(tmp_path):
    z = G.load('fk_raw.npz')
    raw = tmp_path / 'raw'
    raw.mkdir()
    for dst, src in (('train_new.txt', 'val_txt'), ('val_new.txt', 'test_new_txt'), ('test_new.txt', 'test_new_txt'),
                     ('items_a.txt', 'items_a_txt'), ('items_b.txt', 'items_b_txt')):
        (raw / dst).write_bytes(z[src].tobytes())
    return raw


def _args(raw, data):
    return SimpleNamespace(
        dataset='Food-Kitchen', path_raw=str(raw), path_data=str(data), use_raw=True, save_processed=False,
        device=torch.device('cuda:0'), batch_size=128, batch_size_eval=2048, num_workers=0, n_neg_sample=999,
        len_max=15, len_rec=10, d_latent=64, n_gnn=1, n_attn=1, n_head=1, norm_first=False, d_bias=False,
        shared_item_embed=False, dropout_gnn=0.0, dropout_attn=0.0, lr=1e-3, l2=5e-4, lr_step=10, lr_gamma=0.5,
        lambda_loss=0.7, precision='fp32')


def test_food_kitchen_metrics_reproduce(tmp_path):
    from c2dsr_amd.trainer import Trainer
    from oracle.c2dsr_oracle import cal_metrics, cal_score  # utils/metrics.py, which main.py keeps
    ref = G.load('traj_fk.npz')
    random.seed(3407)  # main.py:90-95
    torch.manual_seed(3407)
    torch.cuda.manual_seed_all(3407)
    np.random.seed(3407)
    noter = Noter()
    tr = Trainer(_args(_raw_dir(tmp_path), tmp_path / 'data'), noter)
    sched = torch.optim.lr_scheduler.StepLR(tr.optimizer, step_size=10, gamma=0.5)
    steps = []
    tb = tr.train_batch

    def rec(batch, **kw):
        r = tb(batch, **kw)
        steps.append(torch.stack([x.detach() for x in r]))
        return r

    tr.train_batch = rec
    loader = tr.trainloader
    report = []
    for e in range(int(ref['n_epoch'])):
        order = []

        class Rec:
            dataset = loader.dataset

            def __iter__(self):
                for b in loader:
                    order.append(b[0].numpy().copy())
                    yield b

        tr.trainloader = Rec()
        va, vb = tr.run_epoch()
        sched.step()
        ta, tb_ = tr.run_test()
        np.testing.assert_array_equal(np.concatenate(order), ref[f'e{e}/order_seq_share'], err_msg=f'e{e} order')
        got_steps = torch.stack(steps).cpu().numpy().astype(np.float64)
        steps.clear()
        np.testing.assert_allclose(got_steps, ref[f'e{e}/step_losses'], rtol=1e-4 if e == 0 else 1e-3,
                                   err_msg=f'e{e} step losses')
        report.append((e, 'step_loss_rel', 0, 0, float(np.abs(got_steps / ref[f'e{e}/step_losses'] - 1).max())))
        np.testing.assert_allclose(np.asarray(noter.train[-1]), ref[f'e{e}/loss'], rtol=1e-4, err_msg=f'e{e} loss')
        for k, v in (('val_a', va), ('val_b', vb), ('test_a', ta), ('test_b', tb_)):
            want = ref[f'e{e}/{k}']
            got = np.asarray(v)
            assert got.shape == want.shape, (e, k)
            same = float((got == want).mean())
            near = float((np.abs(got - want) <= 1).mean())
            dm = np.abs(np.asarray(cal_metrics(list(got))) - ref[f'e{e}/{k}_metrics']).max()
            report.append((e, k, same, near, dm))
        report.append((e, 'test_score', 0, 0, float(np.abs(np.asarray(cal_score(ta, tb_, BENCH_FK))
                                                          - ref[f'e{e}/test_score']).max())))
    print('FK (epoch, what, identical ranks, ranks within ±1, max |metric delta|):', report)
    for e, k, same, near, dm in report:
        if k.startswith(('val', 'test_')) and k != 'test_score':
            assert same >= (0.995 if e == 0 else 0.985) and near >= 0.999, (e, k, same, near)
            assert dm <= 1e-3, (e, k, dm)
