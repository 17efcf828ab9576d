"""Drop-in ``trainer.Trainer`` (reference trainer.py:12-181) on the gfx950 path.

Same constructor ``Trainer(args, noter)`` and surface (``run_epoch``, ``run_test``,
``train_batch``, ``evaluate_batch``, ``cal_mask``, ``.model``, ``.optimizer``,
``.scheduler``) so main.py drives it unchanged.  ``train_batch`` runs the model's
HIP forward, the fused loss head (c2dsr_amd/losshead.py), the backward, the
data-parallel gradient all-reduce (RCCL via torch.distributed, when initialised)
and the fused AdamW(amsgrad) step.  Gradients accumulate across the epoch as in
the reference (zero_grad only at the start of run_epoch, Q3).
"""
from __future__ import annotations

import time
from os.path import join

import torch
import torch.distributed as dist

from .dataloader import get_dataloader
from .graph import make_graph
from .losshead import LossHeadFn, LossMeta
from .models.C2DSR import C2DSR
from .optim import FlatAdamW


def dp_rows(B_full, rank, world, dp_split=True, global_rows=None):
    """Rows of a batch this rank trains and where they sit in the global batch.

    dp_split: rank r takes rows [r·⌈B/p⌉, (r+1)·⌈B/p⌉) of the SAME global batch (p ranks reproduce the
    single-device step); otherwise every rank trains its own batch of B rows (weak scaling), placed at
    global rows [r·B, (r+1)·B).  Returns (lo, hi, row_offset, B_global); row_offset feeds the dropout
    index so every rank drops exactly what one device would."""
    if world > 1 and dp_split:
        per = (B_full + world - 1) // world
        lo, hi = min(B_full, rank * per), min(B_full, (rank + 1) * per)
        return lo, hi, lo, B_full
    B_global = global_rows if global_rows is not None else B_full * world
    return 0, B_full, rank * B_full if world > 1 else 0, B_global


def dp_info():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class Trainer(object):
    def __init__(self, args, noter=None, *, data=None, graphs=None):
        """``data`` = (trainloader, valloader, testloader) and ``graphs`` = (adj_share, adj_specific)
        may be given to skip reading ``args.path_raw`` (tests, benchmarks)."""
        if data is None:
            data = get_dataloader(args)
        self.trainloader, self.valloader, self.testloader = data
        if graphs is None:
            graphs = make_graph(args, join(args.path_raw, 'train_new.txt'))
        self.adj_share, self.adj_specific = graphs
        self.model = C2DSR(args, self.adj_share, self.adj_specific).to(args.device)
        self.model.flatten()
        self.optimizer = FlatAdamW(self.model.flat, lr=args.lr, weight_decay=args.l2)
        self.scheduler = torch.optim.lr_scheduler.StepLR(self.optimizer, step_size=args.lr_step, gamma=args.lr_gamma)
        self.noter = noter
        self.n_tr = len(self.trainloader.dataset) if self.trainloader is not None else 0
        self.n_val = len(self.valloader.dataset) if self.valloader is not None else 0
        self.n_te = len(self.testloader.dataset) if self.testloader is not None else 0
        self.device = args.device
        self.d_latent = args.d_latent
        self.n_item_a = args.n_item_a
        self.n_item_b = args.n_item_b
        self.len_rec = args.len_rec
        self.lambda_loss = args.lambda_loss
        self.rank, self.world = dp_info()
        self.dp_split = True  # slice each global batch across data-parallel ranks

    # ------------------------------------------------------------------ training
    def run_epoch(self):
        self.model.train()
        self.optimizer.zero_grad()
        acc = torch.zeros(3, device=self.device)
        t0 = time.time()
        for batch in self.trainloader:
            self.model.convolve_graph()
            loss, loss_rec, loss_mi = self.train_batch(batch)
            acc += torch.stack([loss, loss_rec, loss_mi]) * batch[0].shape[0]  # one sync per epoch (f4)
        acc = (acc / max(self.n_tr, 1)).tolist()
        if self.noter is not None:
            self.noter.log_train(acc[0], acc[1], acc[2], time.time() - t0)
        self.model.eval()
        ra, rb = [], []
        with torch.no_grad():
            self.model.convolve_graph()
            for batch in self.valloader:
                a, b = self.evaluate_batch(batch)
                ra += a
                rb += b
        return ra, rb

    def run_test(self):
        self.model.eval()
        ra, rb = [], []
        with torch.no_grad():
            for batch in self.testloader:
                a, b = self.evaluate_batch(batch)
                ra += a
                rb += b
        return ra, rb

    def cal_mask(self, gt_mask):
        """trainer.py:85-89 (API compatibility; the fused loss head computes the weights itself)."""
        m = gt_mask.float()
        w = m / m.sum(-1, keepdim=True)
        return w.unsqueeze(-1).repeat(1, 1, self.d_latent)

    def loss_meta(self, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, B_global):
        m = self.model
        allreduce = None
        if self.world > 1:
            allreduce = lambda v: dist.all_reduce(v)  # noqa: E731
        return LossMeta(gt_share_a=gt_share_a, gt_share_b=gt_share_b, gt_a=gt_a, gt_b=gt_b, gm_a=gm_a, gm_b=gm_b,
                        n_a=self.n_item_a, n_b=self.n_item_b, R=self.len_rec, lam=self.lambda_loss,
                        Wa=m.classifier_a.weight, ba=m.classifier_a.bias, Wb=m.classifier_b.weight,
                        bb=m.classifier_b.bias, wpad=m.classifier_pad.weight, bpad=m.classifier_pad.bias,
                        Da_w=m.D_a.weight, Da_b=m.D_a.bias, Db_w=m.D_b.weight, Db_b=m.D_b.bias,
                        precision=m.precision, B_global=B_global, allreduce=allreduce)

    def train_batch(self, batch, *, global_rows=None):
        """trainer.py:91-160.  ``batch``: 14 int64 [B, L] tensors (host or device).  Under data
        parallelism each rank trains its slice of the global batch (or, with ``dp_split=False``, its
        own batch; ``global_rows`` then gives the global batch size)."""
        lo, hi, row_offset, B_global = dp_rows(batch[0].shape[0], self.rank, self.world, self.dp_split, global_rows)
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, neg_a,
         neg_b) = [x[lo:hi].to(self.device, non_blocking=True) for x in batch]
        m = self.model
        m.state.row_offset = row_offset
        h_share, hx, hy = m(seq_share, seq_a, seq_b, pos, pos_a, pos_b)
        h_neg_a = m.forward_share(neg_a, pos)
        h_neg_b = m.forward_share(neg_b, pos)
        meta = self.loss_meta(gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, B_global)
        loss, loss_rec, loss_mi = LossHeadFn.apply(h_share, hx, hy, h_neg_a, h_neg_b, meta)
        loss.backward()
        if self.world > 1:
            dist.all_reduce(m.flat.fresh)
        self.optimizer.step()
        return loss, loss_rec, loss_mi

    # ------------------------------------------------------------------ evaluation
    def evaluate_batch(self, batch):
        """trainer.py:162-181: rank of the ground truth among its sampled negatives
        (ties not counted: rank = #(neg > gt) + 1), per domain of the last item."""
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, idx_last_a, idx_last_b, xory_last, gt_last,
         list_neg) = [x.to(self.device) for x in batch]
        h_share, hx, hy = self.model(seq_share, seq_a, seq_b, pos, pos_a, pos_b)
        B, L, d = h_share.shape
        rows = torch.arange(B, device=self.device)
        flag = xory_last[:, 0]
        h_last = h_share[:, -1]
        rank_a, rank_b = [], []
        for dom, hdom, il, clf in ((0, hx, idx_last_a[:, 0], self.model.classifier_a),
                                   (1, hy, idx_last_b[:, 0], self.model.classifier_b)):
            sel = (flag == dom).nonzero().flatten()
            if sel.numel() == 0:
                continue
            q = h_last[sel] + hdom[rows[sel], il[sel]]
            scores = clf(q)
            gt = scores.gather(1, gt_last[sel])
            neg = scores.gather(1, list_neg[sel])
            r = ((neg > gt).sum(1) + 1).tolist()
            (rank_a if dom == 0 else rank_b).extend(r)
        # keep the reference's output order (rows in batch order within each domain)
        return rank_a, rank_b
