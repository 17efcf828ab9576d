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


def test_raw_ops_refuse_undersized_outputs():
    """every buffer a c2dsr_raw op writes is checked against the extent its size arguments
    imply (tools/raw_extents.py) before the launch — an undersized output raises RuntimeError (here on CPU tensors:
    the extent check runs before the device check)."""
    torch.ops.load_library(EXT)
    R = torch.ops.c2dsr_raw
    i64 = torch.zeros(64, dtype=torch.long)
    # embed_fwd writes X [n_rows, d]: 10 rows of 8 need 80 floats
    with pytest.raises(RuntimeError, match='undersized output'):
        R.embed_fwd(i64, i64, 10, 8, None, None, None, None, 1.0, 0, 0, 0.0, 0, torch.zeros(79), 5, 5, None)
    with pytest.raises(RuntimeError, match='must be on the HIP device'):  # the right size gets past the extent check
        R.embed_fwd(i64, i64, 10, 8, None, None, None, None, 1.0, 0, 0, 0.0, 0, torch.zeros(80), 5, 5, None)
    # a view is measured against its storage: a narrow view of a big enough buffer passes the extent check
    big = torch.zeros(200)
    with pytest.raises(RuntimeError, match='must be on the HIP device'):
        R.embed_fwd(i64, i64, 10, 8, None, None, None, None, 1.0, 0, 0, 0.0, 0, big[100:110], 5, 5, None)
    with pytest.raises(RuntimeError, match='undersized output'):
        R.embed_fwd(i64, i64, 10, 8, None, None, None, None, 1.0, 0, 0, 0.0, 0, big[150:], 5, 5, None)
    # strided outputs: rgemm writes C rows with stride ldc
    with pytest.raises(RuntimeError, match='C holds'):
        R.rgemm(4, 16, 32, torch.zeros(128), 32, torch.zeros(1), 0, torch.zeros(3 * 20 + 15), 20, 1.0, 0.0, None, 0,
                0, 0, 0.0, 0, None)
    # workspaces in bytes, optional outputs only when given
    with pytest.raises(RuntimeError, match='workspace holds'):
        R.embed_bwd(i64, i64, 16, 4, torch.zeros(64), 0, 0, 0.0, 0, 1.0, None, 0, None, 0, None,
                    torch.zeros(3, dtype=torch.uint8), 4)
    with pytest.raises(RuntimeError, match='gP holds'):
        R.embed_bwd(i64, i64, 16, 4, torch.zeros(64), 0, 0, 0.0, 0, 1.0, None, 0, torch.zeros(7), 2, None,
                    torch.zeros(4, dtype=torch.uint8), 4)
    with pytest.raises(RuntimeError, match='Up holds'):
        R.ce3_fused_fwd_u(None, None, None, 100, 50, 256, 3, torch.zeros(300), torch.zeros(300),
                          torch.zeros(3 * 100 * 256 - 1), None, None, None, None, None, torch.zeros(100),
                          torch.zeros(100), torch.zeros(100))
    with pytest.raises(RuntimeError, match='vmax holds'):
        R.adamw(*[torch.zeros(16)] * 5, torch.zeros(15), 16, 1e-3, 0.0, 0.9, 0.999, 1e-8, 1, None)


def test_every_written_raw_buffer_has_an_extent_or_a_reason():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'tools'))
    import gen_torch_ops as g
    from raw_extents import EXTENTS, UNCHECKED
    for _, name, params in g.parse():
        op = name[len('c2dsr_'):]
        for pname, _, ptr, decl in params:
            if ptr and pname != 'stream' and not decl.startswith('const ') and pname not in g.HOST_ARRAYS:
                assert pname in EXTENTS.get(op, {}) or pname in UNCHECKED.get(op, {}), (op, pname)
