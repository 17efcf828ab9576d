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

import gc
import os
import sys
import time
from os.path import join

import numpy as np
import torch
import torch.distributed as dist

from .dataloader import get_dataloader
from . import dropout as DK
from . import ops
from ._lib import error_word, lib, stage_ops, stream
from .dp import CommPlan, DPComm, Zero1
from .graph import make_graph
from .losshead import LossHeadFn, LossMeta, ce_kind
from .metrics import RankMetrics
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


def dp_forced():
    """C2DSR_DP_FORCE=1: a process group of ONE rank still runs the data-parallel step (the collectives of dp.py,
    ZeRO-1, the row-sharded GCN) — how a one-GPU box exercises RCCL itself (tests/test_gpu_rccl.py)."""
    return os.environ.get('C2DSR_DP_FORCE', '0') == '1'


def dp_enabled():
    """Whether the step is data parallel: a process group with more than one rank (or one, forced)."""
    return bool(dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or dp_forced()))


def dp_info():
    if dp_enabled():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def device_identity(dev):
    """A string naming the physical device behind ``dev`` on this host: hostname + PCI domain:bus:device + UUID.
    Two ranks with the same identity share one GPU, whatever their HIP_VISIBLE_DEVICES renumbering says."""
    import socket
    pr = torch.cuda.get_device_properties(dev)
    pci = ':'.join(str(getattr(pr, k, '?')) for k in ('pci_domain_id', 'pci_bus_id', 'pci_device_id'))
    return f'{socket.gethostname()}|{pci}|{getattr(pr, "uuid", "")}'


def dp_backend(identities, rank):
    """'nccl' (RCCL) when every rank drives its own GPU, 'gloo' when some ranks share one (RCCL refuses two
    ranks on one device: the one-GPU rehearsal).  ``identities``: device_identity() of every rank, in rank order;
    the rule is global, so every rank reaches the same backend."""
    return 'gloo' if len(set(identities)) < len(identities) else 'nccl'


def init_data_parallel(args):
    """Data parallelism under an UNCHANGED main.py launched by torchrun (BASELINE north_star).

    main.py builds ``args.device = cuda:<--cuda>`` for every process (reference main.py:72-75) and constructs
    ``Trainer(args, noter)`` (main.py:102) without touching torch.distributed.  When the launcher's environment
    says WORLD_SIZE > 1 and no process group exists yet, this runs before the trainer's first device call:
      * the rank's device is ``cuda:LOCAL_RANK`` (``args.device`` is overwritten — main.py's value is the same
        device on every rank), ``torch.cuda.set_device`` makes it current;
      * the process group is RCCL (``'nccl'``, bound to that device) when every rank drives its own GPU, decided
        from the ranks' physical device identities (PCI address + UUID, exchanged over the launcher's rendezvous
        store before the group exists) — NOT from the local device count, which is 1 on a node whose launcher
        gives each rank its own HIP_VISIBLE_DEVICES; only when ranks really share a device (the one-GPU
        rehearsal) is the group gloo, with a warning, since RCCL refuses two ranks on one device; ``--cuda cpu``
        gives gloo on the host (the product path then stops at its first kernel: there is no CPU fallback).
    ``C2DSR_DP_BACKEND`` overrides the backend.  Returns (rank, world) — (0, 1) outside a launcher; a process
    group the caller initialised itself is used as it is."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if (world <= 1 and not dp_forced()) or not dist.is_available() or dist.is_initialized():
        return dp_info()
    rank = int(os.environ['RANK'])
    local = int(os.environ.get('LOCAL_RANK', rank))
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', world))
    backend = os.environ.get('C2DSR_DP_BACKEND')
    dev = torch.device(getattr(args, 'device', 'cpu'))
    kw = {}
    # the launcher's rendezvous store (MASTER_ADDR / MASTER_PORT, or torchrun's agent store): used for the device
    # exchange below and then handed to the process group, so there is one rendezvous
    store, _, _ = next(dist.rendezvous('env://', rank, world))
    if dev.type == 'cuda':
        n_dev = torch.cuda.device_count()  # counts devices without initialising the runtime
        if n_dev < 1:
            raise RuntimeError('data parallel on cuda: no visible device')
        dev = torch.device('cuda', local % n_dev)
        torch.cuda.set_device(dev)
        if backend is None:
            store.set(f'c2dsr/device/{rank}', device_identity(dev))
            ids = [store.get(f'c2dsr/device/{r}').decode() for r in range(world)]
            backend = dp_backend(ids, rank)
            if backend == 'gloo':
                print(f'[c2dsr] WARNING: ranks share a GPU ({ids[rank]}, {n_dev} visible device(s) for '
                      f'{local_world} local ranks): gloo with host staging instead of RCCL', file=sys.stderr,
                      flush=True)
        if backend == 'nccl':
            kw['device_id'] = dev
    else:
        backend = backend or 'gloo'
    args.device = dev
    dist.init_process_group(backend, store=store, rank=rank, world_size=world, **kw)
    print(f'[c2dsr] data parallel: rank {rank}/{world} on {dev} ({backend})', file=sys.stderr, flush=True)
    return rank, world


# all index plans of a step enqueued right behind the propagations in one batched launch set (else: the lookup
# plans after the first CE sweep, each head's target plan after its forward sweep); measured, see DESIGN §8
PLANS_EARLY = __import__('os').environ.get('C2DSR_PLANS_EARLY', '1') == '1'


class Trainer(object):
    def __init__(self, args, noter=None, *, data=None, graphs=None):
        """``data`` = (trainloader, valloader, testloader) and ``graphs`` = (adj_share, adj_specific)
        may be given to skip reading ``args.path_raw`` (tests, benchmarks).  Under torchrun the process group
        and the rank's device are set up here (init_data_parallel), so main.py needs no change."""
        init_data_parallel(args)
        if data is None:
            data = get_dataloader(args)
        self.trainloader, self.valloader, self.testloader = data
        if graphs is None:
            graphs = make_graph(args, join(args.path_raw, 'train_new.txt'))
        self.adj_share, self.adj_specific = graphs
        self.model = C2DSR(args, self.adj_share, self.adj_specific).to(args.device)
        self.rank, self.world = dp_info()
        self.dp = dp_enabled()
        # one device: the backward accumulates straight into the epoch accumulation (no per-step buffer)
        self.model.flatten(align=4 * self.world, direct=not self.dp)
        self.comm_plan, self.zero = None, None
        if self.dp:
            m = self.model
            head = [m.classifier_a.weight, m.classifier_a.bias, m.classifier_b.weight, m.classifier_b.bias,
                    m.classifier_pad.weight, m.classifier_pad.bias, m.D_a.weight, m.D_b.weight]
            if m.D_a.bias is not None:
                head += [m.D_a.bias, m.D_b.bias]
            self.comm_plan = CommPlan(m.flat, [m.embed_i.weight, m.embed_i_a.weight, m.embed_i_b.weight], self.world,
                                      head=head)
            # ZeRO-1: args.zero1 or C2DSR_ZERO1=1
            if getattr(args, 'zero1', False) or os.environ.get('C2DSR_ZERO1', '0') == '1':
                self.zero = Zero1(m.flat, self.comm_plan, self.rank, self.world)
        self.optimizer = FlatAdamW(self.model.flat, lr=args.lr, weight_decay=args.l2, zero=self.zero)
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
        # the last encoder layer's row-wise part on the rows the loss reads (tests compare both layouts)
        self.compact_rows = True
        # last-layer attention on the read rows / padding keys only (ops.RowsQKVAttnFn)
        self.rows_attn = True
        # projection weight gradients grouped per weight across passes (ops.WGradBatch)
        self.batch_wgrad = True
        self.lambda_loss = args.lambda_loss
        self.dp_split = True  # slice each global batch across data-parallel ranks
        self.model.defer_graph = True  # convolve_graph() → launch behind the step's index work (_train_batch)
        # the launch-sizing counts of a step from the batch's host copy (no device read in the step); the device's
        # own counts are checked against them with C2DSR_CHECK_COUNTS=1
        self.host_counts_ok = True
        self.check_counts = os.environ.get('C2DSR_CHECK_COUNTS', '0') == '1'
        if torch.device(self.device).type == 'cuda':
            error_word().zero_()  # a fresh trainer starts with no index error pending on its device

    # ------------------------------------------------------------------ training
    def run_epoch(self):
        self.model.train()
        self.optimizer.zero_grad()
        acc = torch.zeros(3, device=self.device)
        t0 = time.time()
        for batch in self.trainloader:
            self.model.convolve_graph()
            loss, loss_rec, loss_mi = self.train_batch(batch)
            # device-side sums, one sync per epoch (f4)
            lib('c2dsr_loss_accumulate', loss.detach(), loss_rec.detach(), loss_mi.detach(), float(batch[0].shape[0]),
                acc, stream())
        acc = (acc / max(self.n_tr, 1)).tolist()
        self.check_index_errors()  # after the epoch's one sync: free
        if self.noter is not None:
            self.noter.log_train(acc[0], acc[1], acc[2], time.time() - t0)
        self.model.eval()
        with torch.no_grad():
            self.model.convolve_graph()
            return self._evaluate(self.valloader)

    def run_test(self):
        self.model.eval()
        with torch.no_grad():
            return self._evaluate(self.testloader)

    # ------------------------------------------------------------------ index errors (F.embedding / cross_entropy raise)
    def check_batch_indices(self, hb):
        """The reference's lookups raise IndexError on an index outside their table (F.embedding / nn.Embedding,
        models/C2DSR.py:65-67,81, encoders.py:30; F.cross_entropy on a target outside [0, n_item_x] other than the
        ignore index, trainer.py:143-152) before anything is updated.  With the batch's host copy ``hb`` (numpy, batch
        order) the same check runs here, before a launch; without one, the device checks (prepare)."""
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, gt_share_a, gt_share_b, gt_a, gt_b, _, _, neg_a, neg_b) = hb
        m = self.model
        R = self.len_rec
        bits = 0
        for x in (seq_share, seq_a, seq_b, neg_a, neg_b):
            if x.size and (x.min() < 0 or x.max() >= m.n_item):
                bits |= ops.IDX_ERR_ITEM
        for x in (pos, pos_a, pos_b):
            if x.size and (x.min() < 0 or x.max() >= m.attn_share.len_max):
                bits |= ops.IDX_ERR_POS
        for x, n in ((gt_share_a, self.n_item_a), (gt_a, self.n_item_a), (gt_share_b, self.n_item_b),
                     (gt_b, self.n_item_b)):
            t = x[:, -R:]  # the reference reads the last len_rec targets only (trainer.py:126-129)
            if t.size and (t.min() < 0 or t.max() > n):
                bits |= ops.IDX_ERR_TARGET
        if bits:
            raise IndexError(ops.index_error_message(bits))

    def device_index_check(self, batch_dev):
        """c2dsr::index_check over the step's index tensors (device batch, no host copy): returns the error word
        copied after the checks (int32 [1]) for the step's deferred count read (ops.HostCounts err_slot)."""
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, gt_share_a, gt_share_b, gt_a, gt_b, _, _, neg_a, neg_b) = batch_dev
        m = self.model
        L, R = seq_share.shape[1], self.len_rec
        items = [seq_share, seq_a, seq_b, neg_a, neg_b]
        poss = [pos, pos_a, pos_b]
        tg = [(gt_share_a, self.n_item_a), (gt_a, self.n_item_a), (gt_share_b, self.n_item_b), (gt_b, self.n_item_b)]
        idx = items + poss + [t for t, _ in tg]
        hi = [m.n_item] * 5 + [m.attn_share.len_max] * 3 + [n + 1 for _, n in tg]
        cols = [L] * 8 + [min(R, L)] * 4
        bits = [ops.IDX_ERR_ITEM] * 5 + [ops.IDX_ERR_POS] * 3 + [ops.IDX_ERR_TARGET] * 4
        return stage_ops().index_check(idx, hi, cols, bits)

    def check_index_errors(self):
        """Raise IndexError if a lookup of a step since the last check met an index outside its table (the device
        error word of include/c2dsr.h: the kernels read row 0 instead and flag it, the segment sums skip the key,
        and AdamW changes nothing while it is set).  run_epoch calls it at its one host sync; a caller driving
        train_batch on device batches without a host copy calls it at its own."""
        if torch.device(self.device).type != 'cuda':
            return
        w = error_word()
        bits = int(w[0])
        if bits:
            w.zero_()
            raise IndexError(ops.index_error_message(bits))

    def cal_mask(self, gt_mask):
        """trainer.py:85-89 (API compatibility; the fused loss head computes the weights itself)."""
        m = gt_mask.float()
        w = m / m.sum(-1, keepdim=True)
        return w.unsqueeze(-1).repeat(1, 1, self.d_latent)

    def loss_meta(self, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, B_global):
        m = self.model
        allreduce = None
        if self.dp:
            allreduce = lambda v: dist.all_reduce(v)  # noqa: E731
        return LossMeta(gt_share_a=gt_share_a, gt_share_b=gt_share_b, gt_a=gt_a, gt_b=gt_b, gm_a=gm_a, gm_b=gm_b,
                        n_a=self.n_item_a, n_b=self.n_item_b, R=self.len_rec, lam=self.lambda_loss,
                        Wa=m.classifier_a.weight, ba=m.classifier_a.bias, Wb=m.classifier_b.weight,
                        bb=m.classifier_b.bias, wpad=m.classifier_pad.weight, bpad=m.classifier_pad.bias,
                        Da_w=m.D_a.weight, Da_b=m.D_a.bias, Db_w=m.D_b.weight, Db_b=m.D_b.bias,
                        precision=m.precision, B_global=B_global, allreduce=allreduce)

    # encoder passes → which rows the loss reads: bit 1 / 2 = pooled with the a / b weights
    # (trainer.py:101-108, Q5), bit 4 = the last R positions (classifier heads, trainer.py:122-146)
    PASS_ROWS = ((DK.PASS_SHARE, 1 | 2 | 4), (DK.PASS_A, 1 | 4), (DK.PASS_B, 2 | 4), (DK.PASS_NEG0, 1),
                 (DK.PASS_NEG0 + 1, 2))

    def host_counts(self, hb, *, need, pads, ce):
        """The counts ``prepare``'s device kernels produce, from the host copy ``hb`` of the (rank's slice of
        the) batch (numpy arrays in batch order): the five passes' need-set sizes (c2dsr_need_rows: rows
        with a nonzero a / b pooling weight or among the last R positions, per pass code), their padding-row
        counts (c2dsr_pad_rows: seq == idx_pad), and per classifier head the valid targets among the last R
        positions of the shared and the specific sequences (c2dsr_compact_valid: target != n_items).  Pure
        integer counting, so equal to the device's by construction (checked under C2DSR_CHECK_COUNTS=1)."""
        (seq_share, seq_a, seq_b, _, _, _, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, neg_a, neg_b) = hb
        B, L = gm_a.shape
        R = self.len_rec
        out = []
        if need:
            # rows by (a-weight, b-weight) class, apart for the last R positions (bit 4)
            have = (gm_a != 0).view(np.uint8) + 2 * (gm_b != 0).view(np.uint8)
            cls = np.concatenate([np.bincount(have[:, :L - R].ravel(), minlength=4),
                                  np.bincount(have[:, L - R:].ravel(), minlength=4)])
            out += [int(sum(int(cls[h]) for h in range(8) if h & bits)) for _, bits in self.PASS_ROWS]
        if pads:
            pad = int(self.model.attn_share.idx_pad)
            out += [int(np.count_nonzero(x == pad)) for x in (seq_share, seq_a, seq_b, neg_a, neg_b)]
        if ce:
            for ts, tx, n in ((gt_share_a, gt_a, self.n_item_a), (gt_share_b, gt_b, self.n_item_b)):
                out += [int(np.count_nonzero(ts[:, L - R:] != n)), int(np.count_nonzero(tx[:, L - R:] != n))]
        return out

    def count_flags(self, L):
        """Which count groups prepare() produces for a batch of length L: (need sets, padding rows, CE valid rows)."""
        m = self.model
        need = bool(self.compact_rows and m.training and not m.attn_share.norm_first)
        pads = need and self.rows_attn and ops.attn_rows_ok(L, self.d_latent, m.attn_share.n_head)
        ce = ce_kind(m.precision, self.d_latent) is not None
        return need, pads, ce

    def launch_counts(self, host, *, global_rows=None):
        """The launch sizes of a training step on ``host`` (the batch's host arrays) exactly as the step's device
        kernels count them — for a data pipeline that prepares them with the batch (bench.py does, ahead of the
        timed steps) and hands them to train_batch(counts=...)."""
        lo, hi, _, _ = dp_rows(host[0].shape[0], self.rank, self.world, self.dp_split, global_rows)
        hb = tuple(np.asarray(x[lo:hi]) for x in host)
        self.check_batch_indices(hb)  # counts handed to train_batch come with a validated batch
        need, pads, ce = self.count_flags(hb[0].shape[1])
        return self.host_counts(hb, need=need, pads=pads, ce=ce)

    def prepare(self, gm_a, gm_b, gt_share_a, gt_a, gt_share_b, gt_b, seqs=None, host=None, known=None,
                batch_dev=None):
        """Index work the step sizes its launches by, enqueued ahead of the forward with one deferred host
        read of all its counts (ops.HostCounts; nothing waits until the first count is needed):
          * RowSets of the five encoder passes (c2dsr_need_rows), so the last encoder layer runs its
            row-wise part only where the loss looks, and (seqs: the passes' sequences in PASS_ROWS order)
            their padding rows (c2dsr_pad_rows), the only keys its attention can use;
          * per classifier head, the stacked [share; specific] targets of the last R positions
            (c2dsr_rec_targets) and their valid-row compaction (c2dsr_compact_valid) for the fused CE.
        Returns (need: {pass_id: RowSet}, pads: {pass_id: RowSet},
                 ce_pre: [(tcat, idx, inv, tc, (HostCounts, slot)), ...] or None)."""
        ops.require_device(gm_a)  # (no CPU fallback: refused here, before any operator checks shapes)
        m = self.model
        B, L = gm_a.shape
        M, R = B * L, self.len_rec
        dev = gm_a.device
        counts = []
        need_sets = pad_sets = None
        f_need, f_pads, f_ce = self.count_flags(L)
        n = len(self.PASS_ROWS)
        code = sum(bits << (3 * q) for q, (_, bits) in enumerate(self.PASS_ROWS))
        # one stage operator for all of it (c2dsr::step_prepare)
        heads = ((gt_share_a, gt_a, self.n_item_a), (gt_share_b, gt_b, self.n_item_b)) if f_ce else ()
        out = stage_ops().step_prepare(gm_a, gm_b, R, n, code,
                                       list(seqs) if (f_need and seqs is not None and f_pads) else [],
                                       int(m.attn_share.idx_pad), [t for h in heads for t in h[:2]],
                                       [h[2] for h in heads], bool(f_need))
        o = 0
        if f_need:
            idx, inv, cnt, off = out[0:4]
            need_sets = (idx, inv, off)
            counts.append(cnt)
            o = 4
            if seqs is not None and f_pads:
                pidx, pinv, pcnt, poff = out[4:8]
                pad_sets = (pidx, pinv, poff)
                counts.append(pcnt)
                o = 8
        ce = None
        if f_ce:
            ce = []
            for k in range(2):
                tcat, idx_c, inv_c, tc, cnt = out[o + 5 * k:o + 5 * k + 5]
                ce.append((tcat, idx_c, inv_c, tc))
                counts.append(cnt)
        if self.dp:
            s = stream()
            # the global valid-target counts — all the gradient's normalisation needs (trainer.py:143-156,
            # SURVEY.md §8(e)) — reduced ahead of the forward, overlapped with it
            tg = [c[0] for c in ce] if ce is not None else []
            for ts, tx in ((gt_share_a, gt_a), (gt_share_b, gt_b))[len(tg):]:
                t = torch.empty(2 * B * R, device=dev, dtype=torch.int64)
                lib('c2dsr_rec_targets', ts, tx, B, L, R, t, s)
                tg.append(t)
            cvec = torch.zeros(9, device=dev, dtype=torch.float32)  # [8] (loss_mi) is not written here
            lpw = torch.empty(max(1, int(lib.raw('c2dsr_loss_partials_workspace')(B * R))), device=dev,
                              dtype=torch.float32)
            lib('c2dsr_loss_partials', None, tg[0], self.n_item_a, None, tg[1], self.n_item_b, B * R, cvec, lpw, s)
            self.dp_counts = (cvec, dist.all_reduce(cvec, async_op=True))
        if not counts:
            return {}, {}, None
        if not self.host_counts_ok:
            known = None
        elif known is None and host is not None:
            known = self.host_counts(host, need=need_sets is not None, pads=pad_sets is not None, ce=ce is not None)
        err_slot = None
        if known is None and host is None and batch_dev is not None:
            # no host copy: the batch's indices are range-checked on the device and the verdict rides on the
            # count read the step makes anyway (raises IndexError there, before any backward / optimizer launch)
            counts.append(self.device_index_check(batch_dev))
            err_slot = sum(int(c.numel()) for c in counts) - 1
        hc = ops.HostCounts(torch.cat(counts), known=known, check=self.check_counts, err_slot=err_slot)
        need, pads = {}, {}
        base = 0
        for sets, out in ((need_sets, need), (pad_sets, pads)):
            if sets is not None:
                idx, inv, off = sets
                out.update({pid: ops.RowSet(idx[q], inv[q], (hc, base + q), M, off[q])
                            for q, (pid, _) in enumerate(self.PASS_ROWS)})
                base += len(self.PASS_ROWS)
        ce_pre = None
        if ce is not None:
            ce_pre = [c + ((hc, base + 2 * k),) for k, c in enumerate(ce)]
        return need, pads, ce_pre

    def train_batch(self, batch, *, global_rows=None, host=None, counts=None):
        """trainer.py:91-160.  ``batch``: 14 int64 [B, L] tensors (host or device).  Under data
        parallelism each rank trains its slice of the global batch (or, with ``dp_split=False``, its
        own batch; ``global_rows`` then gives the global batch size).  ``host``: the same 14 arrays on the
        host when ``batch`` is already on the device (a batch of host tensors is its own host copy): the
        step's launch sizes are counted from it, so the host never waits on the device inside a step; ``counts``:
        those sizes already counted by the data pipeline (launch_counts).
        Python's cyclic collector is paused while the step is enqueued (a collection in the middle of the
        launch sequence leaves the device idle); it runs after the optimizer launch, under that kernel."""
        if not gc.isenabled():
            return self._train_batch(batch, global_rows=global_rows, host=host, counts=counts)
        gc.disable()
        try:
            return self._train_batch(batch, global_rows=global_rows, host=host, counts=counts)
        finally:
            gc.enable()

    def _train_batch(self, batch, *, global_rows=None, host=None, counts=None):
        lo, hi, row_offset, B_global = dp_rows(batch[0].shape[0], self.rank, self.world, self.dp_split, global_rows)
        if host is None and all(isinstance(x, torch.Tensor) and x.device.type == 'cpu' for x in batch):
            host = batch
        hb = None
        if host is not None and counts is None:
            hb = tuple(np.asarray(x[lo:hi]) for x in host)
            self.check_batch_indices(hb)  # IndexError before anything is enqueued, as the reference's lookups raise
        dev_batch = [x[lo:hi].to(self.device, non_blocking=True) for x in batch]
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, neg_a,
         neg_b) = dev_batch
        m = self.model
        m.state.row_offset = row_offset
        self.dp_counts = None
        need, pads, ce_pre = self.prepare(gm_a, gm_b, gt_share_a, gt_a, gt_share_b, gt_b,
                                          (seq_share, seq_a, seq_b, neg_a, neg_b), host=hb, known=counts,
                                          batch_dev=dev_batch)
        # the GCN forwards of convolve_graph() are enqueued now, behind the index work (and its count copy when the
        # counts are not known on the host: the host then reads them while the device runs the propagations)
        m.launch_graph()
        plans = None
        early = None
        if m.training and PLANS_EARLY and ce_pre is not None:
            # every plan of the step — the eight lookups' and both heads' target plans — in one batched launch set on
            # the side stream right behind the propagations, so none runs beside the loss head's long sweeps
            st = m.state
            pairs = [pr for sq, ps in ((seq_share, pos), (seq_a, pos_a), (seq_b, pos_b), (neg_a, pos), (neg_b, pos))
                     for pr in ((sq, m.n_item), (ps, m.attn_share.len_max))]
            for k, (W, n) in enumerate(((m.classifier_a.weight, self.n_item_a), (m.classifier_b.weight, self.n_item_b))):
                tc, (hc, slot) = ce_pre[k][3], ce_pre[k][4]
                Mv = int(hc[slot]) + int(hc[slot + 1])
                if Mv and W.requires_grad:
                    pairs.append((tc[:Mv], n + 1))
            ops.index_plans(st, pairs)
            early = st
        elif m.training:
            # the embedding backward's sort plans of every pass (side stream), enqueued by the loss head right
            # after its first long CE launch (one launch per radix pass for all eight: c2dsr_index_plans), issued while
            # the device is busy,
            # instead of ahead of the encoder passes, whose first kernels would wait behind them
            st = m.state
            pairs = [pr for sq, ps in ((seq_share, pos), (seq_a, pos_a), (seq_b, pos_b), (neg_a, pos), (neg_b, pos))
                     for pr in ((sq, m.n_item), (ps, m.attn_share.len_max))]
            plans = lambda: ops.index_plans(st, pairs)  # noqa: E731
        m.state.need, m.state.pad_rows, m.state.compact_out = need, pads, bool(need)
        try:
            h_share, hx, hy = m(seq_share, seq_a, seq_b, pos, pos_a, pos_b)
            h_neg_a = m.forward_share(neg_a, pos)
            h_neg_b = m.forward_share(neg_b, pos)
        finally:
            m.state.need, m.state.pad_rows, m.state.compact_out = {}, {}, False
        meta = self.loss_meta(gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, B_global)
        meta.ce_pre = ce_pre
        meta.after_first_ce = plans
        meta.plan_state = early
        if self.dp_counts is not None:
            meta.counts = self.dp_counts
            meta.reduce_async = lambda t: dist.all_reduce(t, async_op=True)  # noqa: E731
        if need:  # the five encoder outputs hold only these rows
            meta.row_sets = tuple(need[pid] for pid, _ in self.PASS_ROWS)
        loss, loss_rec, loss_mi = LossHeadFn.apply(h_share, hx, hy, h_neg_a, h_neg_b, meta)
        if self.dp:
            # the fresh gradient's collectives, each range issued as soon as the backward has made it final
            # (c2dsr_amd/dp.py): dense params under the GCN backwards, each item table per row chunk of its
            # last GCN backward; all-reduce, or reduce-scatter with ZeRO-1
            tables = [m.embed_i.weight, m.embed_i_a.weight, m.embed_i_b.weight]
            m.state.grad_hook = DPComm(m.flat, self.comm_plan, 5, tables, zero=self.zero)
            meta.on_head_grads = m.state.grad_hook.head_done  # issued as the loss head's backward returns
            try:
                self._backward(loss)
            finally:
                hook, m.state.grad_hook = m.state.grad_hook, None
            hook.finish(wait=False)
            self.optimizer.comm = hook.in_order()  # the optimizer waits for each range's sum just before its update
            meta.finish_values()
        else:
            self._backward(loss)
        self.optimizer.step()
        return loss, loss_rec, loss_mi

    def _backward(self, loss):
        """loss.backward() with the projections' weight-gradient products grouped per weight (ops.WGradBatch,
        bf16 mode: flushed by the last embedding backward, or here)."""
        batch = (ops.WGradBatch(5) if self.batch_wgrad and self.model.precision in (ops.BF16, ops.FP32)
                 else None)
        ops.WBATCH = batch
        try:
            loss.backward()
        finally:
            ops.WBATCH = None
        if batch is not None:
            batch.flush()

    # ------------------------------------------------------------------ evaluation
    def eval_ranks(self, batch):
        """Device ranks of one evaluation batch (trainer.py:162-181 on csrc/eval.hip): returns
        (rank int32 [B], xory int64 [B]); row i belongs to domain a iff xory[i] == 0."""
        (seq_share, seq_a, seq_b, pos, pos_a, pos_b, idx_last_a, idx_last_b, xory_last, gt_last,
         list_neg) = [x.to(self.device) for x in batch]
        h_share, hx, hy = self.model(seq_share, seq_a, seq_b, pos, pos_a, pos_b)
        m = self.model
        rank = ops.eval_rank(h_share, hx, hy, idx_last_a, idx_last_b, xory_last, gt_last, list_neg,
                             m.classifier_a.weight, m.classifier_a.bias, m.classifier_b.weight, m.classifier_b.bias)
        return rank, xory_last.reshape(-1)

    @staticmethod
    def _split(ranks, flags):
        r = torch.cat(ranks).tolist() if ranks else []
        f = torch.cat(flags).tolist() if flags else []
        if any(x < 1 for x in r):
            raise IndexError('evaluation index out of range (idx_last / gt / negative item)')
        ra = [x for x, fl in zip(r, f) if fl == 0]
        rb = [x for x, fl in zip(r, f) if fl != 0]
        return ra, rb

    def evaluate_batch(self, batch):
        """trainer.py:162-181: rank of the ground truth among its sampled negatives (ties not counted:
        rank = #(neg > gt) + 1), split by the domain of the last item, rows in batch order."""
        rank, flag = self.eval_ranks(batch)
        out = self._split([rank], [flag])
        self.check_index_errors()  # the sequences' lookups (after _split's sync)
        return out

    def _evaluate(self, loader):
        ranks, flags = [], []
        for batch in loader:
            rank, flag = self.eval_ranks(batch)
            ranks.append(rank)
            flags.append(flag)
        out = self._split(ranks, flags)  # one host sync per evaluation pass
        self.check_index_errors()  # the sequences' lookups
        return out

    def evaluate_metrics(self, loader):
        """Metrics of a whole evaluation pass on the device (cal_metrics per domain, one host sync):
        returns a metrics.RankMetrics (``.values()``, ``.score(benchmark)``)."""
        acc = RankMetrics(self.device)
        self.model.eval()
        with torch.no_grad():
            for batch in loader:
                rank, flag = self.eval_ranks(batch)
                acc.add(rank, flag)
        return acc
