"""Drop-in ``models.C2DSR`` (reference models/C2DSR.py:8-85): same constructor,
attributes, parameter names/initialisation and methods, computed by gfx950 kernels.

``convolve_graph()`` runs the three GCNs (K1) and keeps their outputs as
``hi_share / hi_a / hi_b``; ``forward`` / ``forward_share`` gather-fuse the
embeddings (K2) and run the sequence encoders.  Each training call of
``convolve_graph`` opens a new dropout "step" (keys for the stateless masks).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from .. import dropout as DK
from .. import ops
from ..graph import CSRGraph, DeviceGraph
from .encoders import GCN, SelfAttention, StepState


class Linear(nn.Linear):
    """nn.Linear whose forward runs the MFMA GEMM (classifier_a/b/pad in the reference trainer)."""
    precision = ops.FP32

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, self.precision)


class Bilinear(nn.Bilinear):
    """nn.Bilinear(d, d, 1) whose forward runs on the HIP kernels (D_a / D_b)."""

    def forward(self, x1, x2):
        return ops.BilinearFn.apply(x1.contiguous(), x2.contiguous(), self.weight, self.bias)


def _as_csr(adj, n) -> CSRGraph:
    if isinstance(adj, CSRGraph):
        return adj
    if isinstance(adj, DeviceGraph):
        return adj.host
    if isinstance(adj, torch.Tensor) and adj.is_sparse:  # reference make_graph output (torch COO)
        a = adj.coalesce().cpu()
        r, c = a.indices().numpy()
        v = a.values().numpy().astype(np.float32)
        rowptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
        return CSRGraph(n, rowptr.astype(np.int32), c.astype(np.int32), v)
    raise TypeError(f'unsupported adjacency type {type(adj)}')


class C2DSR(nn.Module):
    def __init__(self, args, adj, adj_specific):
        super().__init__()
        self.args = args
        self.d_latent = args.d_latent
        self.n_item = args.n_item
        self.n_item_a = args.n_item_a
        self.n_item_b = args.n_item_b
        self.adj_share = _as_csr(adj, args.n_item)
        self.adj_specific = _as_csr(adj_specific, args.n_item)

        # parameter creation in the reference's order (same torch RNG draws)
        self.embed_i = nn.Embedding(self.n_item, self.d_latent, padding_idx=self.n_item - 1)
        if args.shared_item_embed:
            self.embed_i_a = self.embed_i
            self.embed_i_b = self.embed_i
        else:
            self.embed_i_a = nn.Embedding(self.n_item, self.d_latent, padding_idx=self.n_item - 1)
            self.embed_i_b = nn.Embedding(self.n_item, self.d_latent, padding_idx=self.n_item - 1)
        self.gnn_share = GCN(args)
        self.gnn_a = GCN(args)
        self.gnn_b = GCN(args)
        self.attn_share = SelfAttention(args)
        self.attn_a = SelfAttention(args)
        self.attn_b = SelfAttention(args)
        self.classifier_a = Linear(self.d_latent, self.n_item_a)
        self.classifier_b = Linear(self.d_latent, self.n_item_b)
        self.classifier_pad = Linear(self.d_latent, 1)
        nn.init.xavier_uniform_(self.classifier_a.weight)
        nn.init.xavier_uniform_(self.classifier_b.weight)
        nn.init.xavier_uniform_(self.classifier_pad.weight)
        nn.init.zeros_(self.classifier_a.bias)
        nn.init.zeros_(self.classifier_b.bias)
        nn.init.zeros_(self.classifier_pad.bias)
        if args.d_bias:
            self.D_a = Bilinear(self.d_latent, self.d_latent, 1, bias=True)
            self.D_b = Bilinear(self.d_latent, self.d_latent, 1, bias=True)
            nn.init.zeros_(self.D_a.bias)
            nn.init.zeros_(self.D_b.bias)
        else:
            self.D_a = Bilinear(self.d_latent, self.d_latent, 1, bias=False)
            self.D_b = Bilinear(self.d_latent, self.d_latent, 1, bias=False)
        nn.init.xavier_uniform_(self.D_a.weight)
        nn.init.xavier_uniform_(self.D_b.weight)

        self._hi = (None, None, None)
        # deferred propagation (convolve_graph → first read) only for a model driven by c2dsr_amd.Trainer, whose
        # step reads the tables right after its index work; a model used on its own propagates at the call, as
        # the reference does (C2DSR.py:59-62)
        self.defer_graph = False
        self._graph_versions = None
        # row-sharded GCN propagation over the data-parallel ranks (ops.RowShard): args.gnn_shard
        # or C2DSR_GNN_SHARD=1, effective when torch.distributed runs more than one rank
        self.gnn_shard = bool(getattr(args, 'gnn_shard', False)) or os.environ.get('C2DSR_GNN_SHARD', '0') == '1'
        self.row_shard = None
        self._tok = (None, None, None)
        self._sink = (None, None, None)
        self.state = StepState(seed=int(getattr(args, 'seed', 0)))
        for i, g in enumerate((self.gnn_share, self.gnn_a, self.gnn_b)):
            g.state = self.state
            g.table = i
        for a in (self.attn_share, self.attn_a, self.attn_b):
            a.state = self.state
        self.flat = None
        self._dev_graphs = None
        self.set_precision(getattr(args, 'precision', 'fp32'))

    # ------------------------------------------------------------------ setup
    def set_precision(self, precision):
        pr = {'bf16': ops.BF16, 'fp32': ops.FP32, 'fp32_exact': ops.FP32_EXACT}.get(precision, precision)
        if pr not in (ops.FP32, ops.BF16, ops.FP32_EXACT):
            raise ValueError(f'precision {precision!r}: expected fp32, bf16 or fp32_exact')
        self.precision = pr
        for a in (self.attn_share, self.attn_a, self.attn_b):
            a.precision = pr
        for c in (self.classifier_a, self.classifier_b):
            c.precision = pr

    def trainable_named_parameters(self):
        """Parameters that receive gradients (the unused encoder_layer template never does, Q15)."""
        return [(n, p) for n, p in self.named_parameters() if '.encoder_layer.' not in n and p.requires_grad]

    def flatten(self, align: int = 4, direct: bool = False):
        """Move every trainable parameter (and its .grad) into the flat HBM store (slices aligned to
        ``align`` floats; data parallel passes 4·world, c2dsr_amd/dp.py)."""
        from ..flat import FlatStore
        dev = self.embed_i.weight.device
        self.flat = FlatStore(self.trainable_named_parameters(), dev, align, direct)
        return self.flat

    def graphs(self):
        dev = self.embed_i.weight.device
        if self._dev_graphs is None or self._dev_graphs[0].rowptr.device != dev:
            self._dev_graphs = (DeviceGraph(self.adj_share, dev), DeviceGraph(self.adj_specific, dev))
        return self._dev_graphs

    def _shard(self):
        from ..trainer import dp_enabled
        if not self.gnn_shard or not dp_enabled():
            return None
        if self.row_shard is None:
            self.row_shard = ops.RowShard(dist.get_rank(), dist.get_world_size())
        return self.row_shard

    def _tables(self):
        self.launch_graph()
        if self.row_shard is not None:
            self.row_shard.wait()  # the all-gathers of the propagated tables (issued by convolve_graph)
        return self._hi

    # the GCN outputs of the last convolve_graph() (C2DSR.py:60-62)
    hi_share = property(lambda self: self._tables()[0])
    hi_a = property(lambda self: self._tables()[1])
    hi_b = property(lambda self: self._tables()[2])

    def new_step(self):
        self.state.step += 1
        self.state.next_share_pass = DK.PASS_NEG0

    # ------------------------------------------------------------------ reference API
    def convolve_graph(self):
        """C2DSR.py:59-62.  The three propagations are enqueued by ``launch_graph``: at the call, or — for a model
        driven by c2dsr_amd.Trainer (``defer_graph``) — at the first read of a table (hi_* / forward) or earlier by
        the trainer, right after its index work, so that work (and the host read of its counts) is queued ahead of
        the GCN kernels instead of behind them (trainer._train_batch).  A deferred launch refuses item-embedding
        weights modified in place since the call (optimizer step, load_state_dict, manual edits)."""
        if self.training:
            self.new_step()
        self._graph_pending = (torch.is_grad_enabled(), self.training)  # the modes of the call, kept for the launch
        self._graph_versions = self._table_versions()
        if not self.defer_graph:
            self.launch_graph()

    def _table_versions(self):
        # torch in-place ops bump _version; the fused optimizer writes through a kernel and bumps WEIGHTS.epoch
        return (ops.WEIGHTS.epoch,) + tuple(w._version for w in (self.embed_i.weight, self.embed_i_a.weight,
                                                                  self.embed_i_b.weight))

    def launch_graph(self):
        pending = getattr(self, '_graph_pending', None)
        if not pending:
            return
        if self._table_versions() != self._graph_versions:
            # the tables would be built from weights the reference's convolve_graph() never saw
            raise RuntimeError('item-embedding weights were modified between convolve_graph() and the first read '
                               'of its tables (deferred propagation, C2DSR.defer_graph); call convolve_graph() again')
        self._graph_pending = None
        grad, train = pending
        g_share, g_spec = self.graphs()
        sh = self._shard()
        mods = (self.gnn_share, self.gnn_a, self.gnn_b)
        modes = [g.training for g in mods]
        for g in mods:
            g.training = train
        try:
            with torch.set_grad_enabled(grad):
                hs, ts, ss = self.gnn_share.propagate(self.embed_i.weight, g_share, shard=sh)
                ha, ta, sa = self.gnn_a.propagate(self.embed_i_a.weight, g_spec, shard=sh)
                hb, tb, sb = self.gnn_b.propagate(self.embed_i_b.weight, g_spec, shard=sh)
        finally:
            for g, t in zip(mods, modes):
                g.training = t
        self._hi = (hs, ha, hb)
        self._tok, self._sink = (ts, ta, tb), (ss, sa, sb)

    def forward(self, seq_share, seq_a, seq_b, pos_share, pos_a, pos_b):
        """C2DSR.py:64-77 → (h_share, hx, hy), each [B, L, d]."""
        self.launch_graph()
        (ts, ta, tb), (ss, sa, sb) = self._tok, self._sink
        h_share = self.attn_share.forward_items(seq_share, pos_share, self.hi_share, ts, self.embed_i.weight, ss,
                                                DK.PASS_SHARE)
        hx = self.attn_a.forward_items(seq_a, pos_a, self.hi_a, ta, self.embed_i_a.weight, sa, DK.PASS_A)
        hy = self.attn_b.forward_items(seq_b, pos_b, self.hi_b, tb, self.embed_i_b.weight, sb, DK.PASS_B)
        return h_share, hx, hy

    def forward_share(self, seq, pos):
        """C2DSR.py:79-85 (shared table + attn_share only)."""
        self.launch_graph()
        pass_id = self.state.next_share_pass
        self.state.next_share_pass += 1
        return self.attn_share.forward_items(seq, pos, self.hi_share, self._tok[0], self.embed_i.weight,
                                             self._sink[0], pass_id)
