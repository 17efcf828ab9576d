"""Drop-in ``models.encoders``: ``GCN`` and ``SelfAttention`` (models/encoders.py:7-48)
with the reference's constructor/forward signatures and parameter names, computed
by the gfx950 kernels (c2dsr_amd/ops.py).

Parameter containers (nn.Embedding / nn.Linear / nn.LayerNorm) are used only to
hold and initialise weights with the reference's names, order and init schemes
(so ``state_dict`` is interchangeable); their forward is never called.
"""
from __future__ import annotations

import copy
import math

import torch
import torch.nn as nn

from .. import dropout as DK
from .. import ops
from ..graph import DeviceGraph


class MultiheadAttentionParams(nn.Module):
    """Weights of nn.MultiheadAttention(d, n_head): in_proj_weight/bias, out_proj.
    Init order as torch: out_proj Linear init, then xavier_uniform_(in_proj_weight),
    zero in_proj_bias and out_proj.bias."""

    def __init__(self, d, n_head):
        super().__init__()
        self.num_heads = n_head
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d))
        self.out_proj = nn.Linear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.in_proj_bias)
        nn.init.zeros_(self.out_proj.bias)


class EncoderLayerParams(nn.Module):
    """Weights of nn.TransformerEncoderLayer(d, n_head, dim_feedforward=d) (encoders.py:23-25)."""

    def __init__(self, d, n_head, d_ff):
        super().__init__()
        self.self_attn = MultiheadAttentionParams(d, n_head)
        self.linear1 = nn.Linear(d, d_ff)
        self.linear2 = nn.Linear(d_ff, d)
        self.norm1 = nn.LayerNorm(d, eps=1e-8)
        self.norm2 = nn.LayerNorm(d, eps=1e-8)


class EncoderParams(nn.Module):
    """nn.TransformerEncoder(layer, n_attn, LayerNorm) parameter layout: deep copies of the layer."""

    def __init__(self, layer, n_attn, d):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(n_attn)])
        self.norm = nn.LayerNorm(d, eps=1e-8)


class StepState:
    """Per-training-step dropout bookkeeping shared by the model's modules."""

    def __init__(self, seed=0):
        self.seed = seed
        self.step = 0
        self.row_offset = 0   # global batch-row offset of this rank (data parallel)
        self.next_share_pass = DK.PASS_NEG0
        self.grad_hook = None  # c2dsr_amd.dp.DPComm while a data-parallel backward runs
        self.plans = {}  # (step, data_ptr, numel, n_keys) -> ops.IndexPlan (sorted on the side stream)
        self.need = {}   # pass_id -> ops.RowSet: rows of the pass the loss reads (set by Trainer.train_batch)
        self.pad_rows = {}  # pass_id -> ops.RowSet: its padding rows, the attention's keys (idem)
        self.compact_out = False  # encoder outputs of such passes stay [n, d] (the loss reads them through rs.inv)

    def keys(self, site):
        return DK.keys(self.seed, self.step, site)


class SelfAttention(nn.Module):
    """models/encoders.py:7-33: pos-emb add + dropout + post/pre-norm TransformerEncoder
    (n_attn layers, FFN width d, ReLU, eps 1e-8) + final LayerNorm, with the causal
    mask and the inverted key-padding mask (seq != pad ⇒ masked, Q1)."""

    def __init__(self, args):
        super().__init__()
        self.idx_pad = args.idx_pad
        self.len_max = args.len_max
        self.d = args.d_latent
        self.n_head = args.n_head
        self.n_attn = args.n_attn
        self.norm_first = args.norm_first
        self.p = args.dropout_attn
        attn_mask = torch.triu(torch.full((args.len_max, args.len_max), float('-inf')), diagonal=1)
        self.register_buffer('attn_mask', attn_mask)
        self.pos_emb = nn.Embedding(args.len_max, args.d_latent)
        self.encoder_layer = EncoderLayerParams(args.d_latent, args.n_head, args.d_latent)
        self.encoder = EncoderParams(self.encoder_layer, args.n_attn, args.d_latent)
        self.precision = ops.FP32
        self.state = StepState()

    # ---- dropout plumbing ----
    def _drop(self, pass_id, layer, kind):
        p = self.p if self.training else 0.0
        if p <= 0.0:
            return 0.0, (0, 0)
        return p, self.state.keys(DK.site_enc(pass_id, layer, kind))

    def encode(self, x, seq, pass_id, link=None):
        """The TransformerEncoder stack on an already embedded + dropped [B, L, d] input.  link: the
        ops.RowsGrad of the embedding that produced x (its input gradient may then stay in compact parts)."""
        B, L, d = x.shape
        rb_rows = self.state.row_offset * L
        rs = self.state.need.get(pass_id) if self.training and not self.norm_first else None
        n_layers = len(self.encoder.layers)
        for li, lay in enumerate(self.encoder.layers):
            at = lay.self_attn
            p_at, k_at = self._drop(pass_id, li, DK.K_ATTN)
            p_sa, k_sa = self._drop(pass_id, li, DK.K_SA)
            p_fm, k_fm = self._drop(pass_id, li, DK.K_FF_MID)
            p_fo, k_fo = self._drop(pass_id, li, DK.K_FF_OUT)

            def sa_block(inp, res=None):
                o = ops.QKVAttnFn.apply(inp.contiguous(), at.in_proj_weight, at.in_proj_bias, seq, self.idx_pad,
                                        self.n_head, p_at, k_at, self.state.row_offset, self.precision, res)
                return ops.linear(o, at.out_proj.weight, at.out_proj.bias, self.precision)

            def ff_block(inp, res=None):
                ff = ops.FFLink(p_fm)
                f = ops.linear(inp, lay.linear1.weight, lay.linear1.bias, self.precision,
                               relu_drop=(k_fm, p_fm, rb_rows), res=res, ff=ff, ff_role='in')
                return ops.linear(f, lay.linear2.weight, lay.linear2.bias, self.precision, ff=ff, ff_role='out')

            if rs is not None and li == n_layers - 1:
                # Last layer, post-norm: everything after the attention is row-wise, and the loss reads only
                # the rows of `rs` (pooled positions, last R positions) — the rest of the layer and the final
                # LayerNorm run on those rows (dropout indices through the row map, so the masks are the
                # full-size run's).
                r1 = ops.ResidualLink(inv=rs.inv)
                xc = ops.gather_rows_nograd(x.reshape(B * L, d), rs)
                ks = self.state.pad_rows.get(pass_id)
                if ks is not None and ops.attn_rows_ok(L, d, self.n_head):
                    # Q only at these rows, K / V only at the padding rows (the only admissible keys, Q1)
                    oc = ops.RowsQKVAttnFn.apply(x.contiguous(), xc, at.in_proj_weight, at.in_proj_bias, seq,
                                                 self.idx_pad, self.n_head, p_at, k_at, self.state.row_offset,
                                                 self.precision, rs, ks, r1, link if li == 0 else None)
                else:
                    o = ops.QKVAttnFn.apply(x.contiguous(), at.in_proj_weight, at.in_proj_bias, seq, self.idx_pad,
                                            self.n_head, p_at, k_at, self.state.row_offset, self.precision, r1)
                    oc = ops.GatherRowsFn.apply(o.reshape(B * L, d), rs)
                sa = ops.linear(oc, at.out_proj.weight, at.out_proj.bias, self.precision)
                x1 = ops.AddLNFn.apply(xc, sa, lay.norm1.weight, lay.norm1.bias, p_sa, k_sa, rb_rows, lay.norm1.eps,
                                       r1, rs.idx)
                r2 = ops.ResidualLink()
                ff = ops.FFLink(p_fm)
                f = ops.linear(x1, lay.linear1.weight, lay.linear1.bias, self.precision,
                               relu_drop=(k_fm, p_fm, rb_rows, rs.idx), res=r2, ff=ff, ff_role='in')
                f2 = ops.linear(f, lay.linear2.weight, lay.linear2.bias, self.precision, ff=ff, ff_role='out')
                nm = self.encoder.norm
                # norm2 and the final norm in one pass each way (the row between them is never stored)
                outc = ops.AddLN2Fn.apply(x1, f2, lay.norm2.weight, lay.norm2.bias, nm.weight, nm.bias, p_fo, k_fo,
                                          rb_rows, lay.norm2.eps, nm.eps, r2, rs.idx)
                # [n, d]: the loss head reads it through rs.inv (Trainer.train_batch passes the row sets)
                return outc if self.state.compact_out else ops.ExpandRowsFn.apply(outc, rs, (B, L, d))
            if self.norm_first:
                y = ops.AddLNFn.apply(x, None, lay.norm1.weight, lay.norm1.bias, 0.0, (0, 0), 0, lay.norm1.eps)
                x = ops.AddDropFn.apply(x, sa_block(y), p_sa, k_sa, rb_rows)
                y = ops.AddLNFn.apply(x, None, lay.norm2.weight, lay.norm2.bias, 0.0, (0, 0), 0, lay.norm2.eps)
                x = ops.AddDropFn.apply(x, ff_block(y), p_fo, k_fo, rb_rows)
            else:
                # x feeds the block's first projection and the LN residual: the LN backward parks its
                # gradient in the link and the projection's dX accumulates onto it (ops.ResidualLink)
                r1 = ops.ResidualLink()
                x = ops.AddLNFn.apply(x, sa_block(x, r1), lay.norm1.weight, lay.norm1.bias, p_sa, k_sa, rb_rows,
                                      lay.norm1.eps, r1)
                r2 = ops.ResidualLink()
                x = ops.AddLNFn.apply(x, ff_block(x, r2), lay.norm2.weight, lay.norm2.bias, p_fo, k_fo, rb_rows,
                                      lay.norm2.eps, r2)
        nm = self.encoder.norm
        return ops.AddLNFn.apply(x, None, nm.weight, nm.bias, 0.0, (0, 0), 0, nm.eps)

    def forward(self, seq, seq_enc, pos, pass_id=None):
        """encoders.py:29-33 on a caller-provided seq_enc [B, L, d] (the training step's fused path is
        ``forward_items``): ``seq_enc += pos_emb(pos)`` mutates the caller's tensor in place as the reference
        does (Q20), then dropout and the encoder stack."""
        if pass_id is None:
            pass_id = DK.PASS_SHARE
        if not seq_enc.is_contiguous():
            raise ValueError('SelfAttention.forward: seq_enc must be contiguous (it is updated in place)')
        p, k = self._drop(pass_id, 0, DK.K_INPUT)
        L = seq_enc.shape[1]
        x = ops.PosAddFn.apply(seq_enc, self.pos_emb.weight, pos)
        if p > 0.0:
            x = ops.DropFn.apply(x, p, k, self.state.row_offset * L)
        return self.encode(x, seq, pass_id)

    def forward_items(self, seq, pos, H, tok, E, sink, pass_id):
        """Fused C2DSR.py:65-71 + encoders.py:29-33: gather (H[seq]+E[seq])·√d + P[pos], dropout, encoder."""
        p, k = self._drop(pass_id, 0, DK.K_INPUT)
        if self.training and not self.norm_first and self.n_attn == 1:
            # the training step's fast path: the whole pass as one stage operator each way (ops.EncoderPassFn)
            rs, ks = self.state.need.get(pass_id), self.state.pad_rows.get(pass_id)
            B, L = seq.shape
            if rs is not None and ks is not None and ops.fused_pass_ok(self.precision, B, L, self.d, self.n_head):
                keys = [k] + [self._drop(pass_id, 0, kind)[1]
                              for kind in (DK.K_ATTN, DK.K_SA, DK.K_FF_MID, DK.K_FF_OUT)]
                outc = ops.EncoderPassFn.apply(tok, E, self.pos_emb.weight, seq, pos, H, self, self.encoder.norm, rs,
                                               ks, keys, p, self.state.row_offset, self.precision, sink,
                                               math.sqrt(self.d))
                return outc if self.state.compact_out else ops.ExpandRowsFn.apply(outc, rs, (B, L, self.d))
        link = ops.RowsGrad() if self.training else None
        x = ops.EmbedFn.apply(tok, E, self.pos_emb.weight, seq, pos, H, math.sqrt(self.d), p, k,
                              self.state.row_offset, sink, self.idx_pad, link)
        return self.encode(x, seq, pass_id, link)


class GCN(nn.Module):
    """models/encoders.py:36-48: mean of [E, A·drop(E), ...] over n_gnn propagation rounds."""

    def __init__(self, args):
        super().__init__()
        self.dropout_gnn = args.dropout_gnn
        self.n_gnn = args.n_gnn
        self.state = StepState()
        self.table = 0
        self.pad_row = args.idx_pad
        self._graph_cache = None

    def _keys(self):
        p = self.dropout_gnn if self.training else 0.0
        return p, [self.state.keys(DK.site_gcn(self.table, k)) if p > 0 else (0, 0) for k in range(self.n_gnn)]

    def _device_graph(self, adj, device):
        """adj as the reference passes it (the torch sparse COO of utils/graph.make_graph), a CSRGraph or a
        DeviceGraph → the DeviceGraph the SpMM runs on (converted once per adjacency object)."""
        if isinstance(adj, DeviceGraph):
            return adj
        hit = self._graph_cache
        if hit is not None and hit[0] is adj and hit[1].rowptr.device == device:
            return hit[1]
        from .C2DSR import _as_csr
        dg = DeviceGraph(_as_csr(adj, adj.shape[0]), device)
        self._graph_cache = (adj, dg)
        return dg

    def forward(self, h, adj):
        """encoders.py:42-48: h [N, d], adj [N, N] (torch sparse COO as make_graph returns it) → H [N, d] =
        mean(h, A·drop(h), …), differentiable w.r.t. h (ops.GCNPropFn)."""
        p, keys = self._keys()
        return ops.GCNPropFn.apply(h, self._device_graph(adj, h.device), self.n_gnn, p, keys)

    def propagate(self, h, adj, sink=None, shard=None):
        """The training step's fused form (C2DSR.convolve_graph): h [N, d], adj a DeviceGraph → (H, token,
        sink); H's gradient arrives through the sink, filled by the embedding lookups of H (ops.GCNFn).
        ``shard``: an ops.RowShard — this rank propagates its block of rows and the blocks are all-gathered."""
        p, keys = self._keys()
        if sink is None:
            sink = ops.GradSink(h.shape[0], h.shape[1], h.device, self.state)
        H, tok = ops.GCNFn.apply(h, self._device_graph(adj, h.device), self.n_gnn, p, keys, self.pad_row, sink,
                                 shard)
        return H, tok, sink
