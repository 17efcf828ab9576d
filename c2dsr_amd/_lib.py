"""Binding of the gfx950 kernel library (``libc2dsr_hip.so``, C ABI in ``include/c2dsr.h``) through its PyTorch
operator library ``libc2dsr_torch.so`` (c2dsr_amd/csrc_torch/):

* ``torch.ops.c2dsr`` — the stage operators the training step runs on (Tensor in / Tensor out, sizes derived from
  the tensors and checked; stage_ops.cpp), reached as ``stage_ops()``;
* ``torch.ops.c2dsr_raw`` — one schema op per C-ABI entry point (pointers as tensors, the ABI's int sizes), reached
  as ``lib(name, *args)`` for the remaining per-kernel calls and ``lib.raw(name)`` for the size / support queries.

Every call enqueues on torch's current HIP stream: the ``stream()`` argument the call sites pass must be that same
current stream (checked: a call naming another stream raises instead of being reordered; the side-stream index plans
switch streams with ``torch.cuda.stream``).  There is deliberately no fallback: if the libraries (or a GPU) are
missing, calls raise, so nothing silently runs on some other path.
"""
from __future__ import annotations

import os
import re

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# C2DSR_LIB_DIR: a directory holding a variant build of both libraries (tools/lib_variant.sh; the operator library
# loads the kernel library next to it)
_DIR = os.environ.get('C2DSR_LIB_DIR') or _HERE
LIB_PATH = os.path.join(_DIR, 'libc2dsr_hip.so')
TORCH_LIB_PATH = os.path.join(_DIR, 'libc2dsr_torch.so')
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'c2dsr.h')


def parse_header(path: str = HEADER) -> dict:
    """name -> (return type, [(param name, is_pointer)]) for every ``c2dsr_*`` declaration."""
    text = open(path).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    out = {}
    for m in re.finditer(r'\b(int|size_t)\s+(c2dsr_\w+)\s*\(([^)]*)\)\s*;', text):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        params = []
        for a in args.split(','):
            a = ' '.join(a.split())
            if a:
                params.append((a.replace('*', ' ').split()[-1], '*' in a))
        out[name] = (ret, params)
    return out


class HipLibError(RuntimeError):
    pass


_ops = {}


def _load_ops():
    """torch.ops.c2dsr / c2dsr_raw, loading libc2dsr_torch.so (and through it libc2dsr_hip.so) once."""
    if not _ops:
        for p in (LIB_PATH, TORCH_LIB_PATH):
            if not os.path.exists(p):
                raise HipLibError(f'{p} not built (run `make` or __graft_entry__.build())')
        torch.ops.load_library(TORCH_LIB_PATH)
        _ops['stage'], _ops['raw'] = torch.ops.c2dsr, torch.ops.c2dsr_raw
    return _ops


def stage_ops():
    """torch.ops.c2dsr (the stage operators; stage_ops.cpp)."""
    return _load_ops()['stage']


class _Lib:
    def __init__(self):
        self._sigs = None
        self._fns = {}  # name -> (raw op, has trailing stream param)
        self.time_meta = {}  # name -> fn(call args): a value appended to that call's timing record (bench accounting)
        self._extra = {}

    def load(self):
        """Load the operator libraries (import check of __graft_entry__.build()); returns the raw op namespace."""
        if self._sigs is None:
            self._sigs = parse_header()
        return _load_ops()['raw']

    @property
    def symbols(self) -> list:
        self.load()
        return sorted(self._sigs)

    def _fn(self, name):
        f = self._fns.get(name)
        if f is None:
            raw = self.load()
            ret, params = self._sigs[name]
            has_stream = bool(params) and params[-1] == ('stream', True)
            f = self._fns[name] = (getattr(raw, name[len('c2dsr_'):]), has_stream)
        return f

    def __call__(self, name: str, *args):
        """One entry point on torch's current stream; tensors (or None) for pointers, numpy arrays for the host
        descriptor arrays, ints / floats for scalars.  Raises HipLibError on a failed launch."""
        op, has_stream = self._fn(name)
        if self.time_meta and name in self.time_meta:
            self._extra.setdefault(name, []).append(self.time_meta[name](args))
        if has_stream:
            # the call sites' stream() argument: the op launches on torch's current stream itself, so a call naming
            # any other stream would be silently reordered — refused instead
            s = args[-1]
            if s is not None and s != torch.cuda.current_stream().cuda_stream:
                raise HipLibError(f'{name}: stream argument {s:#x} is not the current stream (use torch.cuda.stream)')
            args = args[:-1]
        args = [torch.from_numpy(a) if type(a) is np.ndarray else a for a in args]
        try:
            return op(*args)
        except RuntimeError as e:
            raise HipLibError(str(e)) from None

    def raw(self, name: str):
        """The op of a query entry point (no stream: ``*_supported``, workspace sizes), called with its ints."""
        return self._fn(name)[0]

    # ---- in-process event timing of chosen entry points (bench.py): records (ms, args as numbers + extras)
    def timing_start(self, names):
        """Bracket every later call of these entry points (made anywhere: here or inside a stage operator) with HIP
        events on its launch stream; an empty list stops."""
        self._extra = {}
        stage_ops().timing_set(sorted(names))

    def timing_take(self) -> dict:
        """name -> [(ms, [the call's arguments as numbers (pointers as addresses, null 0), extras...])] in launch
        order; a time_meta value of the call (host-side calls only) is appended last."""
        names, ms, meta, lens = stage_ops().timing_take()
        out, o = {}, 0
        for n, t, k in zip(names, ms, lens):
            out.setdefault(n, []).append((t, list(meta[o:o + k])))
            o += k
        for n, vals in self._extra.items():
            for rec, v in zip(out.get(n, []), vals):
                rec[1].append(v)
        self._extra = {}
        return out


lib = _Lib()


def stream() -> int:
    """The current HIP stream (the kernels' launch stream; raises without a device: no CPU fallback)."""
    if not torch.cuda.is_available():
        raise HipLibError('c2dsr_amd kernels need a HIP device (no CPU fallback)')
    return torch.cuda.current_stream().cuda_stream


def error_word() -> torch.Tensor:
    """The current device's index error word (int32 [4], aliased; word 0 holds the C2DSR_IDX_ERR_* bits of
    include/c2dsr.h): every range-checked lookup of a training step ORs into it, AdamW changes nothing while it is
    nonzero, and the trainer reads it at its host sync (Trainer.check_index_errors)."""
    return stage_ops().error_word()


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise HipLibError('c2dsr_amd kernels need tensors on the HIP device (no CPU fallback)')
