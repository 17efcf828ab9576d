"""Bucketed data-parallel gradient all-reduce, overlapped with the backward.

The step has one real exchange: the sum all-reduce of this step's flat gradient
(``FlatStore.fresh``).  Instead of one collective after ``loss.backward()``, the flat
buffer is cut into buckets that become final at known points of the backward, and each
bucket's all-reduce is issued (``async_op=True``: RCCL on its own stream, ordered after
the kernels already enqueued) the moment it is final, so the collectives run under the
remaining backward kernels:

* the **dense** bucket (every parameter that is not an item table: pos_emb, encoder,
  classifier heads, D_a/D_b) is final once the last embedding-lookup backward
  (``EmbedFn.backward``, the tail of every encoder pass) has run — the loss head and
  every encoder backward precede it by data dependence.  It is issued then, under the
  three GCN backwards;
* each **item table** bucket (``embed_i``, ``embed_i_a``, ``embed_i_b``; one bucket when
  ``shared_item_embed``) is final after the last GCN backward that reads that table
  (``GCNFn.backward`` writes ``E.grad`` last), and is issued then, under the next table's
  GCN backward.

Reference behaviour replaced: the single-process ``loss.backward(); optimizer.step()``
of trainer.py:156-158 — with these sums the rank-local step equals the single-device
step (global-count loss normalisation, losshead.LossMeta).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class GradBuckets:
    """Issues the per-bucket all-reduces of ``flat.fresh`` as the backward makes them final.

    tables: the item-table parameters (possibly the same one several times); gcn_uses[i]
    is how many GCN backwards will write tables[i]'s gradient this step; n_lookups the
    number of embedding-lookup passes whose backward must run before the dense bucket is
    final.  ``allreduce(t)`` must return a work handle with ``.wait()`` (default:
    ``dist.all_reduce(t, async_op=True)``)."""

    def __init__(self, flat, tables, n_lookups, allreduce=None):
        self.flat = flat
        self.allreduce = allreduce or (lambda t: dist.all_reduce(t, async_op=True))
        ptr2slice = {p.data_ptr(): (o, n) for _, p, o, n in flat.entries}
        self.table_left = {}
        self.table_range = {}
        for t in tables:
            k = t.data_ptr()
            if k not in ptr2slice:
                raise KeyError('table parameter is not in the flat store')
            self.table_left[k] = self.table_left.get(k, 0) + 1
            o, n = ptr2slice[k]
            self.table_range[k] = (o, o + n)
        # dense bucket = complement of the table ranges, merged into contiguous pieces
        cuts = sorted(self.table_range.values())
        dense, lo = [], 0
        for a, b in cuts:
            if a > lo:
                dense.append((lo, a))
            lo = max(lo, (b + 3) // 4 * 4)
        if lo < flat.numel:
            dense.append((lo, flat.numel))
        self.dense = dense
        self.lookups_left = n_lookups
        self.works = []
        self.issued = []  # (lo, hi) in issue order (tests)

    def _issue(self, lo, hi):
        if hi > lo:
            self.works.append(self.allreduce(self.flat.fresh[lo:hi]))
            self.issued.append((lo, hi))

    def lookup_done(self):
        """One embedding-lookup backward finished (EmbedFn.backward / PosDropFn.backward)."""
        self.lookups_left -= 1
        if self.lookups_left == 0:
            for lo, hi in self.dense:
                self._issue(lo, hi)

    def table_done(self, table):
        """One GCN backward finished writing ``table``'s gradient."""
        k = table.data_ptr()
        if k not in self.table_left:
            return
        self.table_left[k] -= 1
        if self.table_left[k] == 0:
            self._issue(*self.table_range[k])

    def finish(self):
        """Issue whatever was not triggered (e.g. a backward that skipped a pass), then make the
        current stream wait for every collective."""
        if self.lookups_left > 0:
            self.lookups_left = 1
            self.lookup_done()
        for k, left in self.table_left.items():
            if left > 0:
                self.table_left[k] = 0
                self._issue(*self.table_range[k])
        covered = sorted(self.issued)
        pos = 0
        for lo, hi in covered:  # every element reduced exactly once
            if lo != pos:
                raise RuntimeError(f'gradient bucket gap at {pos}..{lo}')
            pos = (hi + 3) // 4 * 4
        if pos < self.flat.numel:
            raise RuntimeError('gradient buckets do not cover the flat store')
        for w in self.works:
            w.wait()
        self.works = []


def notify_lookup(state):
    h = getattr(state, 'grad_hook', None)
    if h is not None:
        h.lookup_done()


def notify_table(state, table):
    h = getattr(state, 'grad_hook', None)
    if h is not None:
        h.table_done(table)
