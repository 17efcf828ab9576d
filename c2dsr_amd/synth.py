"""Synthetic two-domain interaction logs in the reference's raw on-disk format.

The reference reads ``<path_raw>/<mode>_new.txt`` (``dataloader.py:39-58``,
``utils/graph.py:33-47``): one user per line,
``user \t id \t item|ts|date| \t item|ts|date| ...``; items live in the
shared index space (domain A = ``[0, n_a)``, domain B = ``[n_a, n_a+n_b)``)
and are ordered by timestamp (stable) when read.  ``items_{a,b}.txt`` only
matter through their line counts (``dataloader.py:237-252``).

Generator: per-domain Zipf(s) popularity, domain of each
position ~ Bernoulli(0.5), length n ~ U[n_min, L] so position 0 stays pad
after left-padding (Q2), strictly increasing timestamps (``ties=True`` adds
equal timestamps and shuffles the line order to exercise the stable sort).
"""
from __future__ import annotations

import os
from os.path import join

import numpy as np


def zipf_probs(n: int, s: float) -> np.ndarray:
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    return w / w.sum()


def make_sequences(n_users: int, n_a: int, n_b: int, len_max: int, *, seed: int = 1,
                   s: float = 1.2, n_min: int = 6, p_a: float = 0.5) -> list[list[int]]:
    """Item sequences (chronological) in the shared id space."""
    rng = np.random.default_rng(seed)
    pa, pb = zipf_probs(n_a, s), zipf_probs(n_b, s)
    # random permutation so that popular ids are spread over the id range
    perm_a = rng.permutation(n_a)
    perm_b = rng.permutation(n_b) + n_a
    n_min = max(2, min(n_min, len_max))
    lens = rng.integers(n_min, len_max + 1, size=n_users)
    seqs = []
    for n in lens:
        dom = rng.random(n) < p_a
        na, nb = int(dom.sum()), int(n - dom.sum())
        ia = perm_a[rng.choice(n_a, size=na, p=pa)]
        ib = perm_b[rng.choice(n_b, size=nb, p=pb)]
        seq = np.empty(n, dtype=np.int64)
        seq[dom] = ia
        seq[~dom] = ib
        seqs.append(seq.tolist())
    return seqs


def write_raw(path: str, mode: str, seqs: list[list[int]], *, seed: int = 7, ties: bool = False) -> str:
    """Write ``<path>/<mode>_new.txt``.  With ``ties`` some timestamps repeat and
    interactions are written out of chronological order."""
    rng = np.random.default_rng(seed)
    os.makedirs(path, exist_ok=True)
    fn = join(path, f'{mode}_new.txt')
    with open(fn, 'w', encoding='utf-8') as f:
        for u, seq in enumerate(seqs):
            ts = 1_300_000_000 + np.cumsum(rng.integers(0 if ties else 1, 5, size=len(seq))) * 86400
            order = np.arange(len(seq))
            if ties:
                order = rng.permutation(len(seq))
            fields = [f'{seq[i]}|{int(ts[i])}|2013-01-01 08:00:00|' for i in order]
            f.write(f'{u}\t{u * 3 + 1}\t' + '\t'.join(fields) + '\n')
    return fn


def write_items(path: str, n_a: int, n_b: int) -> None:
    os.makedirs(path, exist_ok=True)
    for name, n in (('items_a.txt', n_a), ('items_b.txt', n_b)):
        with open(join(path, name), 'w', encoding='utf-8') as f:
            for i in range(n):
                f.write(f'{i}\tASIN{i:08d}\t{i}\n')


def make_dataset(path: str, n_a: int, n_b: int, len_max: int, n_train: int, n_eval: int,
                 *, seed: int = 1, ties: bool = True, n_min: int = 3) -> None:
    """A complete raw dataset directory (train/val/test + item lists)."""
    write_items(path, n_a, n_b)
    for k, (mode, n) in enumerate((('train', n_train), ('val', n_eval), ('test', n_eval))):
        seqs = make_sequences(n, n_a, n_b, len_max, seed=seed + 101 * k, n_min=n_min)
        write_raw(path, mode, seqs, seed=seed + 7 + k, ties=ties)


def make_flat_sequences(n_users: int, n_a: int, n_b: int, len_max: int, *, seed: int = 1, s: float = 1.2,
                        n_min: int = 6, p_a: float = 0.5) -> tuple[np.ndarray, np.ndarray]:
    """Vectorised generator for the large synthetic configs (10M+10M items,
    ~2M sequences): same distribution as :func:`make_sequences` (Zipf(s) popularity per domain over
    a random permutation of the ids, domain ~ Bernoulli(p_a), length ~ U[n_min, L]) returned flat:
    (items int64 [Σn], offsets int64 [n_users+1])."""
    rng = np.random.default_rng(seed)
    n_min = max(2, min(n_min, len_max))
    lens = rng.integers(n_min, len_max + 1, size=n_users)
    off = np.zeros(n_users + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    tot = int(off[-1])
    dom = rng.random(tot) < p_a
    out = np.empty(tot, dtype=np.int64)
    for is_a, n, base in ((True, n_a, 0), (False, n_b, n_a)):
        cdf = np.cumsum(zipf_probs(n, s))
        cdf /= cdf[-1]
        sel = dom if is_a else ~dom
        k = int(sel.sum())
        rank = np.minimum(np.searchsorted(cdf, rng.random(k), side='right'), n - 1)
        perm = rng.permutation(n)
        out[sel] = perm[rank] + base
    return out, off


def transition_edges_flat(items: np.ndarray, off: np.ndarray, n_item_a: int) -> tuple[np.ndarray, np.ndarray]:
    """graph.transition_edges on flat sequences (vectorised; same edge multiset and emission order):
    share = consecutive pairs within a sequence, specific = consecutive same-domain pairs."""
    seq_id = np.repeat(np.arange(off.size - 1, dtype=np.int64), np.diff(off))
    same = seq_id[1:] == seq_id[:-1]
    share = np.stack([items[:-1][same], items[1:][same]], 1)
    is_a = items < n_item_a
    # per domain: consecutive items of that domain within one sequence, interleaved back into the
    # reference's emission order (position of the later item)
    pos = np.arange(items.size, dtype=np.int64)
    parts = []
    for m in (is_a, ~is_a):
        it, sid, ps = items[m], seq_id[m], pos[m]
        ok = sid[1:] == sid[:-1]
        parts.append((ps[1:][ok], it[:-1][ok], it[1:][ok]))
    ps = np.concatenate([p[0] for p in parts])
    order = np.argsort(ps, kind='stable')
    spec = np.stack([np.concatenate([p[1] for p in parts])[order], np.concatenate([p[2] for p in parts])[order]], 1)
    return share.reshape(-1, 2), spec.reshape(-1, 2)
