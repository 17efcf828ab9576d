"""Which linear1 forward precision passes the C2 / d256 reference steps (fp32 mode)?  Runs those tests with
ops.gemm's linear1 call (the exact fp32 GEMM, relu·dropout epilogue, dropout 0 here) replaced by a float64
emulation of a split product: 'x3' (2 bf16 pieces, hi·hi + lo·hi + hi·lo), 'x6' (3 pieces, every term with
piece-order sum <= 4), or 'f64' (the float64 product, rounded once).  Diagnostic only.
usage: python tools/linear1_emu.py MODE"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import c2dsr_amd.ops as ops  # noqa: E402

MODE = sys.argv[1]
orig = ops.gemm


def pieces(x, n):
    out, r = [], x.double()
    for _ in range(n):
        p = r.float().bfloat16().double()
        out.append(p)
        r = r - p
    return out


def emu(A, B, C, *, M, N, K, transA=0, transB=0, bias=None, relu_drop=None, **kw):
    if relu_drop is None or transA or not transB or kw.get('lda') or kw.get('ldb'):
        return orig(A, B, C, M=M, N=N, K=K, transA=transA, transB=transB, bias=bias, relu_drop=relu_drop, **kw)
    assert relu_drop[1] == 0.0, 'dropout-0 reference steps only'
    a, w = A[:M].double(), B[:N].double()
    if MODE == 'f64':
        y = a @ w.T
    else:
        n = 2 if MODE == 'x3' else 3
        ap, wp = pieces(a, n), pieces(w, n)
        terms = [(0, 0), (1, 0), (0, 1)] if MODE == 'x3' else [(i, j) for i in range(3) for j in range(3) if i + j <= 2]
        y = sum(ap[i] @ wp[j].T for i, j in terms)
    if bias is not None:
        y = y + bias.double()
    C[:M] = torch.relu(y).float()
    return C


ops.gemm = emu
sys.exit(pytest.main(['tests/test_gpu_parity.py', '-k', 'c2_step or d256_step', '-s', '-q', '-p', 'no:cacheprovider']))
