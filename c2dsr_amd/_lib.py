"""ctypes binding of the gfx950 kernel library (``libc2dsr_hip.so``, C ABI in
``include/c2dsr.h``).

The argument types are read from the header itself, so the binding and the
declared ABI cannot drift apart.  Tensors are passed as raw device pointers
(``Tensor.data_ptr()``) and the stream as ``torch.cuda.current_stream().cuda_stream``.

There is deliberately no fallback: if the library (or a GPU) is missing, calls
raise, so nothing silently runs on some other path.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (load torch's HIP runtime first: same soname libamdhip64.so.7)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('C2DSR_LIB') or os.path.join(_HERE, 'libc2dsr_hip.so')
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'c2dsr.h')

_CTYPES = {
    'int': ctypes.c_int,
    'long': ctypes.c_long,
    'float': ctypes.c_float,
    'uint32_t': ctypes.c_uint32,
    'int64_t': ctypes.c_int64,
    'size_t': ctypes.c_size_t,
}


def parse_header(path: str = HEADER) -> dict:
    """name -> (restype, [argtypes]) for every ``c2dsr_*`` declaration."""
    text = open(path).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    out = {}
    for m in re.finditer(r'\b(int|size_t)\s+(c2dsr_\w+)\s*\(([^)]*)\)\s*;', text):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        types = []
        for a in args.split(','):
            a = a.strip()
            if not a:
                continue
            if '*' in a:
                types.append(ctypes.c_void_p)
            else:
                base = a.replace('const ', '').split()[0]
                types.append(_CTYPES[base])
        out[name] = (_CTYPES[ret], types)
    return out


class HipLibError(RuntimeError):
    pass


DEBUG_SYNC = os.environ.get('C2DSR_DEBUG_SYNC', '0') == '1'


class _Lib:
    def __init__(self):
        self._lib = None
        self._sigs = None
        self._fns = {}  # name -> bound ctypes function (argtypes set)
        self.time_names = set()  # entry points bracketed by HIP events (bench.py roofline)
        self.timed = {}
        self.time_meta = {}  # name -> fn(args) evaluated at launch; its value is appended to the record

    def load(self):
        if self._lib is not None:
            return self._lib
        if not os.path.exists(LIB_PATH):
            raise HipLibError(f'{LIB_PATH} not built (run `make` or __graft_entry__.build())')
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        sigs = parse_header()
        for name, (res, args) in sigs.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        self._lib, self._sigs = lib, sigs
        return lib

    @property
    def symbols(self) -> list:
        self.load()
        return sorted(self._sigs)

    def __call__(self, name: str, *args):
        fn = self._fns.get(name)
        if fn is None:
            fn = self._fns[name] = getattr(self.load(), name)
        lib = self._lib
        conv = [a.data_ptr() if isinstance(a, torch.Tensor) else a for a in args]
        if not DEBUG_SYNC and name not in self.time_names:  # the common path: one ctypes call
            rc = fn(*conv)
            if rc != 0:
                raise HipLibError(f'{name} failed with hipError {rc}')
            return rc
        if name in self.time_names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = getattr(lib, name)(*conv)
            e1.record()
            meta = self.time_meta.get(name)
            rec = conv + [meta(conv)] if meta is not None else conv
            self.timed.setdefault(name, []).append((e0, e1, rec))
        elif DEBUG_SYNC:  # C2DSR_DEBUG_SYNC=1: attribute an asynchronous device fault to its entry point
            try:
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                raise HipLibError(f'device fault before {name} (after the previous entry point)') from e
            rc = getattr(lib, name)(*conv)
            try:
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                raise HipLibError(f'device fault in {name} (args {conv})') from e
        else:
            rc = getattr(lib, name)(*conv)
        if rc != 0:
            raise HipLibError(f'{name} failed with hipError {rc}')
        return rc

    def raw(self, name: str):
        fn = self._fns.get(name)
        if fn is None:
            fn = self._fns[name] = getattr(self.load(), name)
        return fn


lib = _Lib()


def stream() -> int:
    if not torch.cuda.is_available():
        raise HipLibError('c2dsr_amd kernels need a HIP device (no CPU fallback)')
    return torch.cuda.current_stream().cuda_stream


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise HipLibError('c2dsr_amd kernels need tensors on the HIP device (no CPU fallback)')
