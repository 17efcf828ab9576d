"""The PyTorch-ROCm extension (c2dsr_amd/libc2dsr_torch.so) loads without a GPU and registers one c2dsr_raw schema op
per C-ABI entry point of include/c2dsr.h, with every buffer the entry point writes declared mutable (Tensor(a!)),
plus the c2dsr:: stage operators (no compute here: tests/test_gpu_torch_ops.py)."""
import os

import pytest
import torch

from c2dsr_amd._lib import parse_header

HERE = os.path.dirname(os.path.abspath(__file__))
EXT = os.path.join(os.path.dirname(HERE), 'c2dsr_amd', 'libc2dsr_torch.so')


def test_every_header_entry_point_is_a_torch_op():
    torch.ops.load_library(EXT)
    names = sorted(parse_header())
    assert int(torch.ops.c2dsr_raw.generated_count()) == len(names)
    for n in names:
        op = getattr(torch.ops.c2dsr_raw, n[len('c2dsr_'):])
        assert op.default._schema.name == 'c2dsr_raw::' + n[len('c2dsr_'):]


def _writes(op):
    return {a.name for a in op.default._schema.arguments if a.alias_info is not None and a.alias_info.is_write}


def test_raw_op_schemas_declare_the_buffers_they_write():
    """an op that writes Y / part / C / gW must say so in its schema, or functionalization and
    torch.compile may drop or reorder it; const pointers stay read-only."""
    torch.ops.load_library(EXT)
    R = torch.ops.c2dsr_raw
    assert _writes(R.gcn_spmm) == {'part', 'Y', 'Y2'}
    assert _writes(R.embed_fwd) == {'X', 'err'}  # err: the index error word (C2DSR_IDX_ERR_*)
    assert _writes(R.adamw) == {'p', 'fresh', 'accum', 'm', 'v', 'vmax'}
    assert _writes(R.rgemm_x3) == {'C'}
    assert _writes(R.ce3_fused_dw) == {'dWp', 'dbp'}
    assert _writes(R.wgemm_multi) == {'dW', 'db', 'part'}
    # every non-const pointer of the header is a mutable argument, every const one is not
    hdr = open(os.path.join(os.path.dirname(HERE), 'include', 'c2dsr.h')).read()
    import re
    text = re.sub(r'/\*.*?\*/', '', hdr, flags=re.S)
    for m in re.finditer(r'\b(?:int|size_t)\s+c2dsr_(\w+)\s*\(([^)]*)\)\s*;', text):
        params = [' '.join(a.split()) for a in m.group(2).split(',') if a.strip()]
        want = {a.replace('*', ' ').split()[-1] for a in params if '*' in a and not a.startswith('const ')} - {'stream'}
        assert _writes(getattr(R, m.group(1))) == want, m.group(1)


def test_torch_op_refuses_host_tensors():
    torch.ops.load_library(EXT)
    x = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match='must be on the HIP device'):
        torch.ops.c2dsr_raw.f32_to_bf16(x, 32, x)
