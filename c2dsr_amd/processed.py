"""The reference's processed on-disk formats, read without executing the file.

The reference stores its processed data as pickles under ``path_data``:
  {train,val,test}.pkl   ``pickle.dump(self.data)`` — lists of per-sequence lists of ints
                         (dataloader.py:26-34)
  graph.pkl              ``pickle.dump((adj_share, adj_specific))`` — two torch sparse COO tensors
                         (utils/graph.py:99-107)
They are written here in the same form (so either implementation reads the other's files) and read
with ``_Restricted``, an unpickler whose ``find_class`` admits only the torch reconstruction helpers
a pickled sparse tensor names (tensor / sparse-tensor rebuild, layout, ``torch.Size``), and routes the storage bytes through
``torch.load(..., weights_only=True)``.  Everything else a pickle could name (any other global,
i.e. anything that would run code) raises ``pickle.UnpicklingError``.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np
import torch


def _storage_from_bytes(b):
    return torch.load(io.BytesIO(b), weights_only=True)


_ALLOWED = {
    ('torch._utils', '_rebuild_tensor_v2'): lambda: torch._utils._rebuild_tensor_v2,
    ('torch._utils', '_rebuild_sparse_tensor'): lambda: torch._utils._rebuild_sparse_tensor,
    ('torch.serialization', '_get_layout'): lambda: torch.serialization._get_layout,
    ('torch.storage', '_load_from_bytes'): lambda: _storage_from_bytes,
    ('torch', 'Size'): lambda: torch.Size,
    ('collections', 'OrderedDict'): lambda: __import__('collections').OrderedDict,
}


class _Restricted(pickle.Unpickler):
    def __init__(self, f, allow_tensors: bool):
        super().__init__(f)
        self.allow_tensors = allow_tensors

    def find_class(self, module, name):
        key = (module, name)
        if self.allow_tensors and key in _ALLOWED:
            return _ALLOWED[key]()
        raise pickle.UnpicklingError(f'processed file names {module}.{name}; only plain data is accepted')


def _check_lists(data, path):
    if not isinstance(data, list):
        raise ValueError(f'{path}: expected a list of sequences, got {type(data).__name__}')
    for row in data[:1]:
        if not isinstance(row, (list, tuple)):
            raise ValueError(f'{path}: expected per-sequence lists')
    return data


def load_lists(path: str):
    """dataloader.py:32-34: the processed rows of one split (lists / tuples / ints only)."""
    if not os.path.exists(path):
        raise FileNotFoundError(f'processed data {path} is missing (run once with --use_raw to create it)')
    with open(path, 'rb') as f:
        return _check_lists(_Restricted(f, allow_tensors=False).load(), path)


def _writer_rank() -> bool:
    """Data parallel: one writer (rank 0) — every rank builds the same lists, concurrent truncating writes of
    one path would race (the reference is single-process)."""
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def _dump_atomic(path: str, obj) -> None:
    """pickle to a temporary file beside ``path`` and rename it over ``path``: a reader never sees a torn file."""
    os.makedirs(os.path.dirname(path) or '.', exist_ok=True)
    tmp = f'{path}.tmp{os.getpid()}'
    with open(tmp, 'wb') as f:
        pickle.dump(obj, f)
    os.replace(tmp, path)


def save_lists(path: str, data) -> None:
    """dataloader.py:28-29 (rank 0 only under data parallelism; atomic replace)."""
    if _writer_rank():
        _dump_atomic(path, data)


def _to_sparse(g):
    r, c, v = g.coo()
    idx = torch.from_numpy(np.vstack([r, c]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(np.asarray(v, dtype=np.float32)), (g.n, g.n)).coalesce()


def save_graph(path: str, g_share, g_spec) -> None:
    """utils/graph.py:101-103: the two normalised adjacencies as torch sparse COO tensors (rank 0 only under
    data parallelism; atomic replace)."""
    if _writer_rank():
        _dump_atomic(path, (_to_sparse(g_share), _to_sparse(g_spec)))


def load_graph(path: str):
    """utils/graph.py:104-106: returns (adj_share, adj_specific) as torch sparse COO tensors."""
    if not os.path.exists(path):
        raise FileNotFoundError(f'processed graph {path} is missing (run once with --use_raw --save_processed)')
    with open(path, 'rb') as f:
        pair = _Restricted(f, allow_tensors=True).load()
    if not (isinstance(pair, tuple) and len(pair) == 2 and all(isinstance(a, torch.Tensor) and a.is_sparse
                                                                 for a in pair)):
        raise ValueError(f'{path}: expected (adj_share, adj_specific) sparse tensors')
    return pair
