"""Per-sequence index / mask construction (a1) and the DataLoader surface.

Mirrors dataloader.py of the reference bit-exactly, including the consumption of
Python's global ``random`` (MT19937) stream — one ``randint`` per position for the
cross-domain negatives, ``random.sample`` for the 999 evaluation negatives — so
that with ``random.seed(3407)`` (main.py:91) the produced lists are identical.

  read_raw            dataloader.py:39-58
  preprocess_train    dataloader.py:60-161   (14 lists of length len_max)
  preprocess_evaluate dataloader.py:163-228  (11 lists)
  get_dataloader      dataloader.py:245-259
Quirks kept: the last same-domain item is dropped when the final target is in the
other domain; B's final-target test is ``> n_a`` (Q13); sequences without an A or
a B target are dropped after their negatives were drawn; B evaluation negatives
come from ``range(n_b - n_a)`` (Q14).
"""
from __future__ import annotations

import os
import random
from os.path import join

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from . import prep, processed
from .graph import read_sequences

TRAIN_FIELDS = ('seq_share', 'seq_a', 'seq_b', 'pos', 'pos_a', 'pos_b', 'gt_share_a', 'gt_share_b', 'gt_a',
                'gt_b', 'gt_mask_a', 'gt_mask_b', 'seq_share_neg_a', 'seq_share_neg_b')
EVAL_FIELDS = ('seq_share', 'seq_a', 'seq_b', 'pos', 'pos_a', 'pos_b', 'idx_last_a', 'idx_last_b', 'xory_last',
               'gt_last', 'list_neg')


def _targets_backwards(seq_dom, pos_dom, last_gt_in_domain, last_gt_local, pad, offset):
    """Walk a domain view from the end (dataloader.py:97-133): returns (gt, mask) and
    edits seq_dom/pos_dom in place when the final item loses its target."""
    n = len(seq_dom)
    gt = [None] * n
    mask = [0] * n
    cur = -1
    for i in range(1, n + 1):
        k = n - i
        if not pos_dom[k]:
            continue
        if cur == -1:
            cur = seq_dom[k] - offset
            if last_gt_in_domain:
                gt[k] = last_gt_local
                mask[k] = 1
            else:
                seq_dom[k] = pad
                pos_dom[k] = 0
        else:
            gt[k] = cur
            mask[k] = 1
            cur = seq_dom[k] - offset
    return gt, mask


def process_train_sequence(u, n_a, n_b, pad, len_max, rng=random):
    """One raw sequence → 14 lists, or None if dropped.  Consumes ``rng`` like the reference."""
    gt = u[1:]
    seq = u[:-1]
    n = len(u)
    pos = list(range(1, n))
    seq_a, pos_a, neg_a = [], [], []
    seq_b, pos_b, neg_b = [], [], []
    ca = cb = 1
    for idx in seq:
        if idx < n_a:
            neg_a.append(idx)
            seq_a.append(idx)
            pos_a.append(ca)
            ca += 1
            neg_b.append(rng.randint(0, n_a - 1))
            seq_b.append(pad)
            pos_b.append(0)
        else:
            neg_a.append(rng.randint(n_a, pad - 1))
            seq_a.append(pad)
            pos_a.append(0)
            neg_b.append(idx)
            seq_b.append(idx)
            pos_b.append(cb)
            cb += 1
    g_a, m_a = _targets_backwards(seq_a, pos_a, gt[-1] < n_a, gt[-1], pad, 0)
    if sum(m_a) == 0:
        return None
    g_b, m_b = _targets_backwards(seq_b, pos_b, gt[-1] > n_a, gt[-1] - n_a, pad, n_a)
    if sum(m_b) == 0:
        return None
    gt_a = [n_a if v is None else v for v in g_a]
    gt_b = [n_b if v is None else v for v in g_b]
    lp = len_max - n + 1
    padl = lambda v, x: [v] * lp + x  # noqa: E731
    gt_full = padl(pad, gt)
    gt_share_a = [v if v < n_a else n_a for v in gt_full]
    gt_share_b = [v - n_a if v >= n_a else n_b for v in gt_full]
    return [padl(pad, seq), padl(pad, seq_a), padl(pad, seq_b), padl(0, pos), padl(0, pos_a), padl(0, pos_b),
            gt_share_a, gt_share_b, padl(n_a, gt_a), padl(n_b, gt_b), padl(0, m_a), padl(0, m_b),
            padl(pad, neg_a), padl(pad, neg_b)]


def process_eval_sequence(u, n_a, n_b, pad, len_max, n_neg, rng=random):
    gt_last = u[-1]
    seq = u[:-1]
    n = len(u)
    pos = list(range(1, n))
    seq_a, pos_a, seq_b, pos_b = [], [], [], []
    ca = cb = 1
    for idx in seq:
        if idx < n_a:
            seq_a.append(idx)
            pos_a.append(ca)
            ca += 1
            seq_b.append(pad)
            pos_b.append(0)
        else:
            seq_a.append(pad)
            pos_a.append(0)
            seq_b.append(idx)
            pos_b.append(cb)
            cb += 1
    lp = len_max - n + 1
    pos, pos_a, pos_b = [0] * lp + pos, [0] * lp + pos_a, [0] * lp + pos_b
    seq, seq_a, seq_b = [pad] * lp + seq, [pad] * lp + seq_a, [pad] * lp + seq_b

    def last_idx(p):
        for i in range(1, len_max + 1):
            if p[-i]:
                return len_max - i
        return -1

    ia, ib = last_idx(pos_a), last_idx(pos_b)
    if gt_last < n_a:
        negs = rng.sample(list(range(gt_last)) + list(range(gt_last + 1, n_a)), n_neg)
        return [seq, seq_a, seq_b, pos, pos_a, pos_b, [ia], [ib], [0], [gt_last], negs]
    local = gt_last - n_a
    negs = rng.sample(list(range(local)) + list(range(local + 1, n_b - n_a)), n_neg)
    return [seq, seq_a, seq_b, pos, pos_a, pos_b, [ia], [ib], [1], [local], negs]


def preprocess_train(seqs, n_a, n_b, len_max, rng=random):
    pad = n_a + n_b
    out = []
    for u in seqs:
        r = process_train_sequence(u, n_a, n_b, pad, len_max, rng)
        if r is not None:
            out.append(r)
    return out


def preprocess_evaluate(seqs, n_a, n_b, len_max, n_neg, rng=random):
    pad = n_a + n_b
    return [process_eval_sequence(u, n_a, n_b, pad, len_max, n_neg, rng) for u in seqs]


def to_arrays(rows) -> list[np.ndarray]:
    """list of per-sequence rows → one int64 array per field (rows must be rectangular)."""
    if not rows:
        return []
    return [np.asarray([r[j] for r in rows], dtype=np.int64) for j in range(len(rows[0]))]


def native_prep() -> bool:
    """The native pipeline (c2dsr_amd/prep.py) processes raw files unless C2DSR_PREP=python."""
    return os.environ.get('C2DSR_PREP', 'native') != 'python' and prep.available()


class CDSRDataset(Dataset):
    """dataloader.py:9-37,230-234.  ``args.use_raw`` (main.py:24) selects the source as in the reference:
    raw ``{mode}_new.txt`` under ``path_raw`` (processed here, then saved to ``path_data/{mode}.pkl`` like
    dataloader.py:26-29), else the processed ``path_data/{mode}.pkl`` (dataloader.py:32-34), read with a
    restricted unpickler that accepts only lists, tuples and ints (``processed.load_lists``).  ``args``
    without a ``use_raw`` attribute (tests, benchmarks) read the raw files and write nothing.

    Raw files are processed by the native pipeline (libc2dsr_prep.so, bit-exact, same draws from
    Python's ``random``) or, with C2DSR_PREP=python, by the Python restatement above.  The rows are held
    as one int64 array per field (``fields``); ``data`` gives the reference's list-of-lists form."""

    def __init__(self, args, mode):
        self.mode = mode
        use_raw = getattr(args, 'use_raw', None)
        if use_raw is False:
            self.fields = to_arrays(processed.load_lists(join(args.path_data, mode + '.pkl')))
        else:
            fn = join(args.path_raw, mode + '_new.txt')
            if not os.path.exists(fn):
                raise FileNotFoundError(f'raw {mode} file {fn} is missing (use_raw reads path_raw/{mode}_new.txt)')
            self.fields = self._process(fn, args, mode)
        self.length = len(self.fields[0]) if self.fields else 0
        if use_raw:
            processed.save_lists(join(args.path_data, mode + '.pkl'), self.data)

    @staticmethod
    def _process(fn, args, mode):
        if native_prep():
            rf = prep.RawFile(fn)
            if mode == 'train':
                rows = rf.train_rows(args.n_item_a, args.n_item_b, args.len_max)
                return [rows[:, j] for j in range(rows.shape[1])]
            seqs, last, neg = rf.eval_rows(args.n_item_a, args.n_item_b, args.len_max, args.n_neg_sample)
            return [seqs[:, j] for j in range(6)] + [last[:, j:j + 1] for j in range(4)] + [neg]
        seqs = read_sequences(fn)
        if mode == 'train':
            return to_arrays(preprocess_train(seqs, args.n_item_a, args.n_item_b, args.len_max))
        return to_arrays(preprocess_evaluate(seqs, args.n_item_a, args.n_item_b, args.len_max, args.n_neg_sample))

    @property
    def data(self):
        """The reference's form: one list of per-field lists per sequence."""
        return [[f[i].tolist() for f in self.fields] for i in range(self.length)]

    def __len__(self):
        return self.length

    def __getitem__(self, index):
        return tuple(torch.from_numpy(f[index]) for f in self.fields)


def count_item(path):
    with open(path, 'r', encoding='utf-8') as f:
        return sum(1 for _ in f)


def get_dataloader(args):
    """dataloader.py:245-259: sets n_item_a/b, n_item, idx_pad on args (item counts from ``path_raw`` with
    ``use_raw``, else from ``path_data``, like dataloader.py:247)."""
    p = args.path_data if getattr(args, 'use_raw', None) is False else args.path_raw
    args.n_item_a = count_item(join(p, 'items_a.txt'))
    args.n_item_b = count_item(join(p, 'items_b.txt'))
    args.n_item = args.n_item_a + args.n_item_b + 1
    args.idx_pad = args.n_item - 1
    nw = getattr(args, 'num_workers', 0)
    tr = DataLoader(CDSRDataset(args, 'train'), batch_size=args.batch_size, shuffle=True, num_workers=nw)
    va = DataLoader(CDSRDataset(args, 'val'), batch_size=args.batch_size_eval, shuffle=False, num_workers=nw)
    te = DataLoader(CDSRDataset(args, 'test'), batch_size=args.batch_size_eval, shuffle=False, num_workers=nw)
    return tr, va, te
