"""Diagnostic: worst relative errors of the fp32 mode's d=256 step vs the oracle (tests/test_gpu_parity.py's
C256 case, dropout 0.2, two steps), with the split-bf16 GEMMs everywhere and with linear1's forward (the
ReLU producer) on the exact fp32-input GEMM — to see whether ReLU-boundary sign flips of the pre-activation
explain the gradient residual.  usage: python tools/fp32_diag.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from c2dsr_amd import ops  # noqa: E402
from tests import test_gpu_parity as T  # noqa: E402


def run(tag):
    tr, orc, rows = T._oracle_case(T.C256, B=96, n_users=260, precision='fp32')
    worst = T._steps_vs_oracle(tr, orc, rows, 96, 2, 1.0, 0.05, 1.0)
    top = sorted(worst.items(), key=lambda x: -x[1])[:10]
    print(tag, {k: f'{v:.2e}' for k, v in top}, flush=True)


run('x3 everywhere:')
orig_fwd = ops.LinearFn.forward
orig_kind = ops.rg_kind


def fwd(ctx, x, W, b, precision, relu_drop, *a, **k):
    if relu_drop is not None:
        ops.rg_kind = lambda *q: None
    try:
        return orig_fwd(ctx, x, W, b, precision, relu_drop, *a, **k)
    finally:
        ops.rg_kind = orig_kind


ops.LinearFn.forward = staticmethod(fwd)
run('linear1 forward exact:')
