"""Dropout keys for the stateless counter-hash masks used by the HIP kernels.

The reference samples torch-CPU Bernoulli masks (F.dropout / nn.Dropout in
models/encoders.py:20,45 and inside nn.TransformerEncoderLayer), which no GPU RNG
can reproduce.  Here every dropout *site* of a training step gets a key pair
(k0, k1) derived from (seed, step, site); the kernels hash the element index with
it (include/c2dsr.h), so a mask costs no memory and the backward regenerates it.
Element indices of activation dropouts use the GLOBAL batch row, so data-parallel
ranks drop exactly what a single device would for the same global batch.
"""
from __future__ import annotations

_M64 = (1 << 64) - 1


def _mix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def keys(seed: int, step: int, site: int) -> tuple[int, int]:
    x = _mix64((seed & _M64) ^ _mix64((step * 0x100000001B3 + site) & _M64))
    return x & 0xFFFFFFFF, x >> 32


# ---- site ids --------------------------------------------------------------
GCN_TABLES = {'share': 0, 'a': 1, 'b': 2}
# encoder passes within one train step: forward() → share/a/b, forward_share() → 3, 4, ...
PASS_SHARE, PASS_A, PASS_B, PASS_NEG0 = 0, 1, 2, 3
K_INPUT, K_ATTN, K_SA, K_FF_MID, K_FF_OUT = 0, 1, 2, 3, 4


def site_gcn(table: int, layer: int) -> int:
    return 0x100 + table * 16 + layer


def site_enc(pass_id: int, layer: int, kind: int) -> int:
    return 0x1000 + pass_id * 256 + (0 if kind == K_INPUT else 1 + layer * 8 + (kind - 1))
