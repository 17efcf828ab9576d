"""Data-parallel gradient exchange, overlapped with the backward.

The step has one real exchange: the sum over ranks of this step's flat gradient
(``FlatStore.fresh``).  ``CommPlan`` cuts the flat store, once, into *reduction ranges* that become
final at known points of the backward; ``DPComm`` issues each range's collective (``async_op=True``:
RCCL on its own stream, ordered after the kernels already enqueued) the moment it is final, so the
collectives run under the remaining backward kernels:

* the **head** range (classifier_a/b/pad, D_a/D_b: ≈26 M of the MB config's 106 M parameters) is final
  when the loss head's backward returns (nothing else reads those parameters) and is issued then, under
  the five encoder backwards;
* the **dense** ranges (pos_emb and the encoders) are final once the last embedding-lookup backward
  (``EmbedFn.backward``, the tail of every encoder pass) has run and are issued then, under the three
  GCN backwards;
* each **item table** (``embed_i``, ``embed_i_a``, ``embed_i_b``; one table when ``shared_item_embed``)
  is final after the last GCN backward that reads it.  A table's GCN backward runs as soon as the last
  lookup of its propagated table has run its backward (``ops.GradSink.lookup_done``; autograd alone would
  run all three after every other node): table B's after pass B, table A's after pass A — their collectives
  run under the backward of the passes after them — and the share table's after the last share pass.  Its
  last SpMM runs in row chunks (``ops.gcn_backward`` asks ``row_cuts``) and each chunk's collective is
  issued as soon as the chunk is written — so only the last chunk of the share table is exposed.

Two modes:
  ``allreduce``  every rank ends with the summed gradient in ``fresh`` and runs the (replicated) AdamW
                 over all of it (c2dsr_amd/optim.py);
  ``zero1``      ZeRO-1: each range is reduce-scattered, rank r receiving the sum of its 1/p part of the
                 range into ``Zero1.gshard``; AdamW updates only the owned parts (optimizer state and the
                 epoch accumulation are 1/p-sized), then each range's parameters are all-gathered
                 (``Zero1.gather``).  Same bytes on the wire as the all-reduce (reduce-scatter +
                 all-gather), 1/p of the optimizer's HBM traffic and state.

Every range's length is a multiple of 4·world elements (FlatStore aligns every parameter slice to
4·world), so the reduce-scatter splits it into equal float4-aligned parts.

Reference behaviour replaced: the single-process ``loss.backward(); optimizer.step()`` of
trainer.py:156-158 — with these sums the rank-local step equals the single-device step (global-count
loss normalisation, losshead.LossMeta).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

TABLE_CHUNKS = 4  # row chunks of the last GCN backward of each table (collectives issued per chunk)
ROW_ALIGN = 8     # chunk boundaries at multiples of 8 rows


class CommPlan:
    """Static partition of ``flat`` into reduction ranges.

    tables: item-table parameters (possibly the same one several times: shared_item_embed).
    Attributes: ``dense`` [(lo, hi)], ``table_chunks`` {table ptr: [(r0, r1, lo, hi)]} (rows r0..r1 of the
    table ↔ flat range lo..hi; the last chunk also covers the slice's alignment padding), ``ranges`` every
    range in a fixed order (dense first, then the tables' chunks), ``index`` {(lo, hi): position}."""

    def __init__(self, flat, tables, world: int, chunks: int = TABLE_CHUNKS, head=()):
        """head: parameters whose gradient is final when the loss head's backward returns (their slices,
        merged where contiguous, become ``head`` ranges issued then)."""
        self.world = world
        align = 4 * world
        ptr2 = {p.data_ptr(): (o, n, p) for _, p, o, n in flat.entries}
        self.table_chunks = {}
        cuts = []
        for t in tables:
            k = t.data_ptr()
            if k in self.table_chunks:
                continue
            if k not in ptr2:
                raise KeyError('table parameter is not in the flat store')
            o, n, p = ptr2[k]
            N, d = p.shape
            hi = o + flat.padded(n)
            if (o % align) or (hi % align):
                raise ValueError('flat store is not aligned for this world size')
            rows = sorted({min(N, (N * c // chunks) // ROW_ALIGN * ROW_ALIGN) for c in range(chunks)} | {N})
            if (ROW_ALIGN * d) % align:
                rows = [0, N]  # chunk boundaries would not be aligned: one chunk
            ch = []
            for a, b in zip(rows[:-1], rows[1:]):
                if b > a:
                    ch.append((a, b, o + a * d, hi if b == N else o + b * d))
            self.table_chunks[k] = ch
            cuts.append((o, hi))
        tab = sorted(cuts)
        hs = sorted({(ptr2[p.data_ptr()][0], ptr2[p.data_ptr()][0] + flat.padded(ptr2[p.data_ptr()][1]))
                     for p in head if p.data_ptr() in ptr2 and p.data_ptr() not in self.table_chunks})
        self.head = []
        for a, b in hs:  # merge contiguous head slices
            if self.head and self.head[-1][1] == a:
                self.head[-1] = (self.head[-1][0], b)
            else:
                self.head.append((a, b))
        dense, lo = [], 0
        for a, b in sorted(tab + self.head):
            if a > lo:
                dense.append((lo, a))
            lo = max(lo, b)
        if lo < flat.numel:
            dense.append((lo, flat.numel))
        self.dense = dense
        self.ranges = list(self.head) + list(dense) + [(lo, hi) for ch in self.table_chunks.values()
                                                       for _, _, lo, hi in ch]
        self.index = {r: i for i, r in enumerate(self.ranges)}
        pos = 0
        for lo, hi in sorted(self.ranges):  # every element in exactly one range
            if lo != pos or (hi - lo) % align:
                raise RuntimeError(f'reduction ranges do not tile the flat store at {pos}..{lo}')
            pos = hi
        if pos != flat.numel:
            raise RuntimeError('reduction ranges do not cover the flat store')


def _gloo_cuda(t):
    return t.is_cuda and dist.get_backend() == 'gloo'


def reduce_scatter(out, inp):
    """Sum of ``inp`` over ranks, this rank's 1/world part into ``out`` (async handle).  gloo (CPU
    rehearsal of several ranks on one device) has no device reduce-scatter: all-reduce a copy instead."""
    if _gloo_cuda(inp):
        tmp = inp.clone()
        dist.all_reduce(tmp)
        r, n = dist.get_rank(), out.numel()
        out.copy_(tmp[r * n:(r + 1) * n])
        return _Done()
    return dist.reduce_scatter_tensor(out, inp, async_op=True)


def all_gather(out, inp):
    """Every rank's ``inp`` (its part of ``out``, possibly a view of it) into ``out`` (async handle)."""
    if _gloo_cuda(inp):
        parts = [torch.empty_like(inp) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, inp.clone())
        out.copy_(torch.cat(parts))
        return _Done()
    return dist.all_gather_into_tensor(out, inp, async_op=True)


class _Done:
    def wait(self):
        pass


class Zero1:
    """ZeRO-1 ownership: rank r owns the r-th 1/world part of every reduction range.  The owned parts,
    concatenated in ``plan.ranges`` order, form this rank's shard (``shard_numel`` elements); the
    optimizer keeps its state and the epoch accumulation only for the shard."""

    def __init__(self, flat, plan: CommPlan, rank: int, world: int, gather=None):
        self.flat, self.plan, self.rank, self.world = flat, plan, rank, world
        self.parts = []  # (range lo, range hi, own lo, own hi, shard offset)
        off = 0
        for lo, hi in plan.ranges:
            c = (hi - lo) // world
            self.parts.append((lo, hi, lo + rank * c, lo + (rank + 1) * c, off))
            off += c
        self.shard_numel = off
        self.gshard = torch.zeros(off, device=flat.device, dtype=torch.float32)
        self._gather = gather or all_gather

    def part_of(self, rng):
        return self.parts[self.plan.index[rng]]

    def gather(self):
        """All-gather every range's updated parameters (owned part → all ranks); returns the handles."""
        p = self.flat.param
        return [self._gather(p[lo:hi], p[olo:ohi]) for lo, hi, olo, ohi, _ in self.parts]


class DPComm:
    """Issues the collectives of one backward as the backward makes each range final.

    n_lookups: the embedding-lookup passes whose backward must run before the dense ranges are final;
    gcn_uses: {table ptr: GCN backwards that read it this step}.  ``reduce(rng)`` launches one range's
    collective and returns a handle with ``.wait()`` (defaults: all-reduce of ``fresh[lo:hi]``, or with
    ``zero`` a reduce-scatter into the owned part of ``zero.gshard``)."""

    def __init__(self, flat, plan: CommPlan, n_lookups, tables, zero: Zero1 | None = None, reduce=None):
        self.flat, self.plan, self.zero = flat, plan, zero
        if reduce is None:
            if zero is None:
                reduce = lambda lo, hi: dist.all_reduce(flat.fresh[lo:hi], async_op=True)  # noqa: E731
            else:
                def reduce(lo, hi):
                    _, _, olo, ohi, off = zero.part_of((lo, hi))
                    return reduce_scatter(zero.gshard[off:off + ohi - olo], flat.fresh[lo:hi])
        self.reduce = reduce
        self.lookups_left = n_lookups
        self.table_left = {}
        for t in tables:
            k = t.data_ptr()
            self.table_left[k] = self.table_left.get(k, 0) + 1
        self.done = [False] * len(plan.ranges)
        self.works = []
        self.issued = []  # (lo, hi) in issue order (tests)
        self.work_of = {}  # (lo, hi) -> its collective's handle

    def _issue(self, lo, hi):
        i = self.plan.index[(lo, hi)]
        if not self.done[i]:
            self.done[i] = True
            w = self.reduce(lo, hi)
            self.works.append(w)
            self.issued.append((lo, hi))
            self.work_of[(lo, hi)] = w

    def head_done(self):
        """The loss head's backward returned: the classifier / discriminator gradients are final."""
        for lo, hi in self.plan.head:
            self._issue(lo, hi)

    def lookup_done(self):
        """One embedding-lookup backward finished (EmbedFn.backward / PosDropFn.backward)."""
        self.lookups_left -= 1
        if self.lookups_left == 0:
            for lo, hi in self.plan.dense:
                self._issue(lo, hi)

    def row_cuts(self, table):
        """Row chunks [(r0, r1)] for the GCN backward about to write ``table``'s gradient if it is that
        table's last one this step (its collectives then go per chunk), else None."""
        k = table.data_ptr()
        if self.table_left.get(k) != 1:
            return None
        return [(r0, r1) for r0, r1, _, _ in self.plan.table_chunks[k]]

    def table_rows_done(self, table, r0, r1):
        """Rows r0..r1 of ``table``'s gradient are final (a chunk of its last GCN backward)."""
        for a, b, lo, hi in self.plan.table_chunks[table.data_ptr()]:
            if r0 <= a and b <= r1:
                self._issue(lo, hi)

    def table_done(self, table):
        """One GCN backward finished writing ``table``'s gradient."""
        k = table.data_ptr()
        if k not in self.table_left:
            return
        self.table_left[k] -= 1
        if self.table_left[k] == 0:
            for _, _, lo, hi in self.plan.table_chunks[k]:
                self._issue(lo, hi)

    def finish(self, wait=True):
        """Issue whatever was not triggered (e.g. a backward that skipped a pass), then make the current
        stream wait for every collective — or (wait=False) leave the waits to the consumer: ``in_order()``."""
        for lo, hi in self.plan.ranges:
            self._issue(lo, hi)
        if wait:
            for w in self.works:
                w.wait()
            self.works, self.work_of = [], {}

    def in_order(self):
        """[(lo, hi, handle)] of every range in issue order, for a consumer that waits range by range: the
        optimizer updates the ranges whose sums have landed while the last ones are still on the wire
        (FlatAdamW.step)."""
        out = [(lo, hi, self.work_of[(lo, hi)]) for lo, hi in self.issued]
        self.works, self.work_of = [], {}
        return out


def notify_lookup(state):
    h = getattr(state, 'grad_hook', None)
    if h is not None:
        h.lookup_done()


def notify_table(state, table):
    h = getattr(state, 'grad_hook', None)
    if h is not None:
        h.table_done(table)


def row_cuts(state, table):
    h = getattr(state, 'grad_hook', None)
    return None if h is None else h.row_cuts(table)


def notify_rows(state, table, r0, r1):
    h = getattr(state, 'grad_hook', None)
    if h is not None:
        h.table_rows_done(table, r0, r1)
