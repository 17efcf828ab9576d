"""ctypes binding of the native data pipeline (include/c2dsr_prep.h, c2dsr_amd/libc2dsr_prep.so).

``RawFile(path)`` parses a raw ``{mode}_new.txt`` once; ``.train_rows`` / ``.eval_rows`` build the
reference's per-sequence index arrays (dataloader.py:60-228) and ``.edges`` the transition edges
(utils/graph.py:54-81), all bit-exact with the Python restatement in dataloader.py / graph.py and
consuming Python's global ``random`` stream exactly as the reference does: the MT19937 state is read
with ``random.getstate()`` and written back with ``random.setstate()``."""
from __future__ import annotations

import ctypes
import os
import random

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libc2dsr_prep.so')
_lib = None
_i64p = ctypes.POINTER(ctypes.c_int64)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f'{LIB_PATH} is not built (make -C <repo> c2dsr_amd/libc2dsr_prep.so)')
        L = ctypes.CDLL(LIB_PATH)
        L.c2dsr_prep_open.restype = ctypes.c_void_p
        L.c2dsr_prep_open.argtypes = [ctypes.c_char_p]
        L.c2dsr_prep_close.argtypes = [ctypes.c_void_p]
        L.c2dsr_prep_sizes.argtypes = [ctypes.c_void_p, _i64p, _i64p]
        L.c2dsr_prep_sequences.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.c2dsr_prep_train.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, _i64p]
        L.c2dsr_prep_eval.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.c2dsr_prep_edges.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _i64p, ctypes.c_void_p, _i64p]
        L.c2dsr_prep_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def available() -> bool:
    return os.path.exists(LIB_PATH)


def _check(rc):
    if rc != 0:
        raise ValueError(lib().c2dsr_prep_error().decode())


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class _PyRandomState:
    """Python's global MT19937 state as the uint32[625] the library advances in place."""

    def __enter__(self):
        v, st, self.gauss = random.getstate()
        if v != 3 or len(st) != 625:
            raise RuntimeError('unexpected random.getstate() layout')
        self.st = np.asarray(st, dtype=np.uint32)
        return self.st

    def __exit__(self, exc_type, *_):
        if exc_type is None:
            random.setstate((3, tuple(int(x) for x in self.st), self.gauss))
        return False


class RawFile:
    def __init__(self, path: str):
        self.h = None
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.h = lib().c2dsr_prep_open(path.encode())
        if not self.h:
            raise ValueError(f'{path}: {lib().c2dsr_prep_error().decode()}')
        n, m = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().c2dsr_prep_sizes(self.h, ctypes.byref(n), ctypes.byref(m)))
        self.n_seq, self.n_items = n.value, m.value

    def close(self):
        if self.h:
            lib().c2dsr_prep_close(self.h)
            self.h = None

    __del__ = close

    def sequences(self):
        """(offsets [n_seq+1], items [n_items]) int64, items of each line in timestamp order."""
        off = np.empty(self.n_seq + 1, dtype=np.int64)
        items = np.empty(max(self.n_items, 1), dtype=np.int64)
        _check(lib().c2dsr_prep_sequences(self.h, _ptr(off), _ptr(items)))
        return off, items[:self.n_items]

    def train_rows(self, n_a: int, n_b: int, len_max: int) -> np.ndarray:
        """dataloader.py:60-161: int64 [rows, 14, len_max] (dropped sequences removed)."""
        out = np.empty((max(self.n_seq, 1), 14, len_max), dtype=np.int64)
        n = ctypes.c_int64()
        with _PyRandomState() as st:
            _check(lib().c2dsr_prep_train(self.h, n_a, n_b, len_max, _ptr(st), _ptr(out), ctypes.byref(n)))
        return out[:n.value]

    def eval_rows(self, n_a: int, n_b: int, len_max: int, n_neg: int):
        """dataloader.py:163-228: (seqs [n, 6, L], last [n, 4] = idx_last_a/b, xory, gt, neg [n, n_neg])."""
        n = self.n_seq
        seqs = np.empty((max(n, 1), 6, len_max), dtype=np.int64)
        last = np.empty((max(n, 1), 4), dtype=np.int64)
        neg = np.empty((max(n, 1), n_neg), dtype=np.int64)
        with _PyRandomState() as st:
            _check(lib().c2dsr_prep_eval(self.h, n_a, n_b, len_max, n_neg, _ptr(st), _ptr(seqs), _ptr(last),
                                         _ptr(neg)))
        return seqs[:n], last[:n], neg[:n]

    def edges(self, n_a: int):
        """utils/graph.py:54-81: (share [E, 2], specific [E', 2]) int64 in emission order."""
        m = max(self.n_items, 1)
        share = np.empty((m, 2), dtype=np.int64)
        spec = np.empty((m, 2), dtype=np.int64)
        ns, npp = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().c2dsr_prep_edges(self.h, n_a, _ptr(share), ctypes.byref(ns), _ptr(spec), ctypes.byref(npp)))
        return share[:ns.value], spec[:npp.value]
