"""The operator library (c2dsr_amd/libc2dsr_torch.so: c2dsr_raw:: and the stage ops the training step uses) runs the
same kernels as a direct ctypes call of the C ABI (the binding INTEGRATION.md §3 shows a maintainer would add): a GCN
SpMM round with dropout, the embedding gather and a split-bf16 projection, each called both ways on the same inputs
— bit-identical outputs."""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'
EXT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'c2dsr_amd', 'libc2dsr_torch.so')


@pytest.fixture(scope='module', autouse=True)
def _ext():
    from c2dsr_amd._lib import lib
    lib.load()
    torch.ops.load_library(EXT)
    yield


_CT = {'int': ctypes.c_int, 'long': ctypes.c_long, 'float': ctypes.c_float, 'uint32_t': ctypes.c_uint32,
       'int64_t': ctypes.c_int64, 'size_t': ctypes.c_size_t}


def _cabi(name):
    """c2dsr_<name> of libc2dsr_hip.so through ctypes, argument types from include/c2dsr.h; tensors → data_ptr,
    the current stream appended."""
    import re
    from c2dsr_amd._lib import HEADER, LIB_PATH
    text = re.sub(r'/\*.*?\*/', '', open(HEADER).read(), flags=re.S)
    m = re.search(r'\bint\s+c2dsr_' + name + r'\s*\(([^)]*)\)\s*;', text)
    types = []
    for a in m.group(1).split(','):
        a = a.strip()
        types.append(ctypes.c_void_p if '*' in a else _CT[a.replace('const ', '').split()[0]])
    f = getattr(ctypes.CDLL(LIB_PATH), 'c2dsr_' + name)
    f.restype, f.argtypes = ctypes.c_int, types

    def call(*args):
        conv = [a.data_ptr() if isinstance(a, torch.Tensor) else a for a in args]
        assert f(*conv, torch.cuda.current_stream().cuda_stream) == 0
    return call


def test_torch_ops_equal_ctypes_path():
    from c2dsr_amd.graph import CSRGraph, DeviceGraph
    from c2dsr_amd.ops import rgemm, to_split_bf16
    T = torch.ops.c2dsr_raw
    g = torch.Generator().manual_seed(11)
    # GCN SpMM (one propagation round: mask on the gathered rows, mean epilogue) over a Zipf-ish graph
    n, d = 3000, 256
    rows = np.sort(np.random.default_rng(3).integers(0, n, 9000))
    cols = np.random.default_rng(4).zipf(1.3, 9000).clip(1, n) - 1
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=rp[1:])
    val = np.random.default_rng(5).random(9000).astype(np.float32)
    dg = DeviceGraph(CSRGraph(n, rp.astype(np.int32), cols.astype(np.int32), val), torch.device(DEV))
    work, n_work, split, n_split, n_slots, col, v = dg.plan(False)
    part = torch.empty(max(1, n_slots), d, device=DEV)
    X = torch.randn(n, d, generator=g).to(DEV)
    outs = []
    for way in ('ctypes', 'torch'):
        Y = torch.empty(n, d, device=DEV)
        args = (work, n_work, split, n_split, part, col, v, d, X, 7, 9, 0.2, 0, 0.5, X, 0.5, 0.0, -1, 0.0, Y, None)
        if way == 'ctypes':
            _cabi('gcn_spmm')(*args)
        else:
            T.gcn_spmm(*args)
        outs.append(Y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    # embedding gather (H[seq] + E[seq])·√d + P[pos], input dropout
    B, L = 64, 50
    seq = torch.randint(0, n, (B, L), generator=g).to(DEV)
    pos = torch.randint(0, L, (B, L), generator=g).to(DEV)
    P = torch.randn(L, d, generator=g).to(DEV)
    outs = []
    for way in ('ctypes', 'torch'):
        Xo = torch.empty(B * L, d, device=DEV)
        args = (seq, pos, B * L, d, X, X, None, P, 16.0, 3, 4, 0.2, 0, Xo, n, L, None)
        if way == 'ctypes':
            _cabi('embed_fwd')(*args)
        else:
            T.embed_fwd(*args)
        outs.append(Xo)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    # split-bf16 projection (fp32 mode) with bias
    M, N, K = 1000, 256, 256
    A, W, b = torch.randn(M, K, generator=g).to(DEV), torch.randn(N, K, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    Wx = to_split_bf16(W)
    C0 = rgemm(A, Wx, torch.empty(M, N, device=DEV), M=M, N=N, K=K, bias=b, x3=True)
    C1 = torch.empty(M, N, device=DEV)
    _cabi('rgemm_x3')(M, N, K, A, K, Wx, 2 * K, C1, N, 1.0, 0.0, b, 0, 0, 0, 0.0, 0, None, 0, None, None, 0.0)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)
