"""Trainer.host_counts (the step's launch sizes counted from the batch's host copy, so the host never reads a count
back from the device inside a step) against a per-element restatement of the device kernels' set predicates
(csrc/loss.hip NeedOp / PadOp / ValidOp).  Equality with the device's own counts is checked on the GPU
(tests/test_gpu_parity.py::test_host_counts_equal_device_counts and the full-size cases, C2DSR_CHECK_COUNTS)."""
from types import SimpleNamespace

import numpy as np

from c2dsr_amd.trainer import Trainer


def _loop_counts(hb, L, R, pad, n_a, n_b, pass_rows):
    (seq_share, seq_a, seq_b, _, _, _, gt_share_a, gt_share_b, gt_a, gt_b, gm_a, gm_b, neg_a, neg_b) = hb
    B = gm_a.shape[0]
    need = []
    for _, bits in pass_rows:  # NeedOp::mask
        k = 0
        for b in range(B):
            for l in range(L):
                have = int(gm_a[b, l] != 0) | (int(gm_b[b, l] != 0) << 1) | (int(l >= L - R) << 2)
                k += (have & bits) != 0
        need.append(k)
    pads = [int(sum(x[b, l] == pad for b in range(B) for l in range(L))) for x in (seq_share, seq_a, seq_b, neg_a, neg_b)]
    ce = []
    for ts, tx, n in ((gt_share_a, gt_a, n_a), (gt_share_b, gt_b, n_b)):  # rec_targets + ValidOp (ignore = n)
        tcat = [ts[b, L - R + r] for b in range(B) for r in range(R)] + [tx[b, L - R + r] for b in range(B) for r in range(R)]
        BR = B * R
        ce += [sum(t != n for t in tcat[:BR]), sum(t != n for t in tcat[BR:])]
    return need + pads + ce


def test_host_counts_match_kernel_predicates():
    rng = np.random.default_rng(7)
    B, L, R, n_a, n_b = 24, 12, 4, 30, 40
    pad = n_a + n_b
    arrs = []
    for k in range(14):
        if k in (10, 11):  # gm_a, gm_b: 0/1 masks
            arrs.append((rng.random((B, L)) < 0.4).astype(np.int64))
        elif k in (6, 8):  # share / specific targets of domain a (ignore index n_a)
            arrs.append(rng.integers(0, n_a + 1, size=(B, L)).astype(np.int64))
        elif k in (7, 9):
            arrs.append(rng.integers(0, n_b + 1, size=(B, L)).astype(np.int64))
        else:  # sequences / positions with padding
            x = rng.integers(0, pad + 1, size=(B, L)).astype(np.int64)
            x[:, : L // 3] = pad
            arrs.append(x)
    fake = SimpleNamespace(PASS_ROWS=Trainer.PASS_ROWS, len_rec=R, n_item_a=n_a, n_item_b=n_b,
                           model=SimpleNamespace(attn_share=SimpleNamespace(idx_pad=pad)))
    got = Trainer.host_counts(fake, tuple(arrs), need=True, pads=True, ce=True)
    want = _loop_counts(tuple(arrs), L, R, pad, n_a, n_b, Trainer.PASS_ROWS)
    assert got == [int(v) for v in want]
    # subsets keep the device order: need sets, then padding rows, then (Mv0, Mv1) per head
    assert Trainer.host_counts(fake, tuple(arrs), need=False, pads=False, ce=True) == got[10:]
    assert Trainer.host_counts(fake, tuple(arrs), need=True, pads=False, ce=False) == got[:5]


def test_host_counts_refuse_a_length_mismatch():
    """counts prepared under other flags than the step's would be read from the wrong slots."""
    import pytest
    import torch
    from c2dsr_amd.ops import HostCounts
    hc = HostCounts(torch.zeros(4, dtype=torch.int32), known=[1, 2, 3, 4])
    assert [hc[i] for i in range(4)] == [1, 2, 3, 4]
    with pytest.raises(ValueError, match='host-prepared counts'):
        HostCounts(torch.zeros(14, dtype=torch.int32), known=[1, 2, 3, 4])
