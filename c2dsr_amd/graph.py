"""Item-transition graphs (a2): the operand of the GCN SpMM.

Mirrors utils/graph.py:33-109 of the reference (``preprocess_graph`` / ``normalize`` /
``make_graph``), built straight into CSR (and the CSR of Aᵀ for the backward)
instead of a torch sparse COO:

* each raw line ``user \\t id \\t item|ts|...`` is stable-sorted by timestamp (:36-47);
* ``adj_share`` gets an edge pre→d for every consecutive pair, ``adj_specific``
  an edge src→d between consecutive same-domain items (A: d < n_a, else B) (:54-81).
  The reference's de-dup dictionary is never filled (Q11), so repeated
  transitions are all kept and summed: edge weight = transition count;
* rows are normalised D⁻¹A with 1/deg computed in float32 by np.power(rowsum, -1)
  and zero-degree rows left 0 (:10-17, :86-92), value = fl32(r_inv[i] * count).
"""
from __future__ import annotations

import codecs
import os
from dataclasses import dataclass

import numpy as np
import torch


def read_sequences(filename: str) -> list[list[int]]:
    """dataloader.py:39-58 / utils/graph.py:36-47: items of each line, stable-sorted by timestamp."""
    out = []
    with codecs.open(filename, 'r', encoding='utf-8') as f:
        for line in f:
            fields = line.strip().split('\t')[2:]
            pairs = []
            for w in fields:
                parts = w.split('|')
                pairs.append((int(parts[0]), int(parts[1])))
            pairs.sort(key=lambda e: e[1])
            out.append([p[0] for p in pairs])
    return out


def transition_edges(seqs: list[list[int]], n_item_a: int) -> tuple[np.ndarray, np.ndarray]:
    """(share_edges [E,2], specific_edges [E',2]) in the reference's emission order."""
    share, spec = [], []
    for seq in seqs:
        src = tgt = pre = -1
        for d in seq:
            if d < n_item_a:
                if src != -1:
                    spec.append((src, d))
                src = d
            else:
                if tgt != -1:
                    spec.append((tgt, d))
                tgt = d
            if pre != -1:
                share.append((pre, d))
            pre = d
    return np.asarray(share, dtype=np.int64).reshape(-1, 2), np.asarray(spec, dtype=np.int64).reshape(-1, 2)


@dataclass
class CSRGraph:
    n: int
    rowptr: np.ndarray  # int32 [n+1]
    col: np.ndarray     # int32 [nnz]
    val: np.ndarray     # float32 [nnz]

    @property
    def nnz(self) -> int:
        return int(self.col.size)

    def transpose(self) -> 'CSRGraph':
        rows = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.rowptr))
        order = np.lexsort((rows, self.col))
        col_t = rows[order].astype(np.int32)
        val_t = self.val[order]
        cnt = np.bincount(self.col, minlength=self.n)
        rowptr = np.zeros(self.n + 1, dtype=np.int64)
        np.cumsum(cnt, out=rowptr[1:])
        return CSRGraph(self.n, rowptr.astype(np.int32), col_t, val_t)

    def coo(self):
        rows = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.rowptr))
        return rows, self.col.astype(np.int64), self.val


def normalized_csr(edges: np.ndarray, n: int) -> CSRGraph:
    """Count-weighted, row-normalised adjacency (utils/graph.py:10-17,86-92)."""
    if edges.size == 0:
        return CSRGraph(n, np.zeros(n + 1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32))
    key = edges[:, 0] * n + edges[:, 1]
    uk, cnt = np.unique(key, return_counts=True)  # sorted by (row, col)
    row = uk // n
    col = uk % n
    deg = np.bincount(edges[:, 0], minlength=n).astype(np.float32)  # exact integer row sums
    with np.errstate(divide='ignore'):
        r_inv = np.power(deg, np.float32(-1)).astype(np.float32)
    r_inv[np.isinf(r_inv)] = np.float32(0.0)
    val = (r_inv[row] * cnt.astype(np.float32)).astype(np.float32)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(row, minlength=n), out=rowptr[1:])
    return CSRGraph(n, rowptr.astype(np.int32), col.astype(np.int32), val)


def preprocess_graph(seqs_or_file, n_item_a: int, n_item: int) -> tuple[CSRGraph, CSRGraph]:
    """A raw file is parsed and walked by the native pipeline (c2dsr_amd/prep.py) unless
    C2DSR_PREP=python; a list of sequences by :func:`transition_edges`."""
    from . import prep
    if isinstance(seqs_or_file, str) and os.environ.get('C2DSR_PREP', 'native') != 'python' and prep.available():
        e_share, e_spec = prep.RawFile(seqs_or_file).edges(n_item_a)
        return normalized_csr(e_share, n_item), normalized_csr(e_spec, n_item)
    seqs = read_sequences(seqs_or_file) if isinstance(seqs_or_file, str) else seqs_or_file
    e_share, e_spec = transition_edges(seqs, n_item_a)
    return normalized_csr(e_share, n_item), normalized_csr(e_spec, n_item)


SPLIT = 64  # max edges per SpMM work item (Zipf-popular items are cut into pieces)


def work_plan(g: CSRGraph, split: int = SPLIT):
    """Static load-balancing plan of the SpMM kernel (include/c2dsr.h:c2dsr_gcn_spmm):
    work [n_work, 4] = (row, e_begin, e_end, slot), split [n_split, 4] = (row, slot_b, slot_e, 0)."""
    deg = np.diff(g.rowptr.astype(np.int64))
    pieces = np.maximum(1, (deg + split - 1) // split)
    n_work = int(pieces.sum())
    row = np.repeat(np.arange(g.n, dtype=np.int64), pieces)
    first = np.repeat(np.cumsum(pieces) - pieces, pieces)
    k = np.arange(n_work, dtype=np.int64) - first  # piece index within its row
    eb = g.rowptr[row].astype(np.int64) + k * split
    ee = np.minimum(eb + split, g.rowptr[row + 1].astype(np.int64))
    is_split = pieces[row] > 1
    slot = np.full(n_work, -1, dtype=np.int64)
    slot[is_split] = np.arange(int(is_split.sum()))
    work = np.stack([row, eb, ee, slot], 1).astype(np.int32)
    srows = np.nonzero(pieces > 1)[0]
    sp = pieces[srows]
    sb = np.cumsum(sp) - sp
    split_arr = np.stack([srows, sb, sb + sp, np.zeros_like(srows)], 1).astype(np.int32)
    return work, split_arr, int(is_split.sum())


class DeviceGraph:
    """CSR of A and of Aᵀ resident on the device (buffers owned by the model), with the
    SpMM work plans of both."""

    def __init__(self, g: CSRGraph, device):
        self.n = g.n
        self.nnz = g.nnz
        t = g.transpose()
        to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        self.rowptr, self.col, self.val = to(g.rowptr), to(g.col), to(g.val)
        self.rowptr_t, self.col_t, self.val_t = to(t.rowptr), to(t.col), to(t.val)
        w, s, nslot = work_plan(g)
        wt, st, nslot_t = work_plan(t)
        self.work, self.split, self.n_work, self.n_split, self.n_slots = to(w), to(s), len(w), len(s), nslot
        self.work_t, self.split_t, self.n_work_t, self.n_split_t, self.n_slots_t = (to(wt), to(st), len(wt), len(st),
                                                                                    nslot_t)
        self.host = g
        self._rowptr_t_host = t.rowptr
        self._row_keys = {False: (w[:, 0], s[:, 0]), True: (wt[:, 0], st[:, 0])}  # host copies, sorted by row

    def row_slice(self, transposed: bool, r0: int, r1: int):
        """(w0, w1, s0, s1): the work items and split combines of output rows r0..r1."""
        wr, sr = self._row_keys[transposed]
        w0, w1 = np.searchsorted(wr, [r0, r1])
        s0, s1 = np.searchsorted(sr, [r0, r1])
        return int(w0), int(w1), int(s0), int(s1)

    def host_rowptr(self, transposed: bool):
        return self._rowptr_t_host if transposed else self.host.rowptr

    def plan(self, transposed: bool):
        if transposed:
            return self.work_t, self.n_work_t, self.split_t, self.n_split_t, self.n_slots_t, self.col_t, self.val_t
        return self.work, self.n_work, self.split, self.n_split, self.n_slots, self.col, self.val

    def to_torch_sparse(self):
        r, c, v = self.host.coo()
        return torch.sparse_coo_tensor(np.vstack([r, c]), v, (self.n, self.n))


def make_graph(args, filename: str):
    """utils/graph.py:99-109.  With ``args.use_raw`` (or no such attribute) the graphs are built from the
    raw train file (and saved to ``path_data/graph.pkl`` when ``args.save_processed``); with
    ``use_raw=False`` they are read from that file (processed.load_graph: no code runs from it)."""
    from . import processed
    use_raw = getattr(args, 'use_raw', None)
    if use_raw is False:
        a_s, a_p = processed.load_graph(os.path.join(args.path_data, 'graph.pkl'))
        from .models.C2DSR import _as_csr
        return _as_csr(a_s, args.n_item), _as_csr(a_p, args.n_item)
    if not os.path.exists(filename):
        raise FileNotFoundError(f'raw train file {filename} is missing (the graph is built from it)')
    g_share, g_spec = preprocess_graph(filename, args.n_item_a, args.n_item)
    if use_raw and getattr(args, 'save_processed', False):
        processed.save_graph(os.path.join(args.path_data, 'graph.pkl'), g_share, g_spec)
    return g_share, g_spec
