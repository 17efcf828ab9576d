"""The PyTorch-ROCm extension (c2dsr_amd/libc2dsr_torch.so, TORCH_LIBRARY(c2dsr)) loads without a GPU and
registers one schema op per C-ABI entry point of include/c2dsr.h (no compute: that is tests/test_gpu_torch_ops.py)."""
import os

import torch

from c2dsr_amd._lib import parse_header

HERE = os.path.dirname(os.path.abspath(__file__))
EXT = os.path.join(os.path.dirname(HERE), 'c2dsr_amd', 'libc2dsr_torch.so')


def test_every_header_entry_point_is_a_torch_op():
    torch.ops.load_library(EXT)
    names = sorted(parse_header())
    assert int(torch.ops.c2dsr.generated_count()) == len(names)
    for n in names:
        op = getattr(torch.ops.c2dsr, n[len('c2dsr_'):])
        assert op.default._schema.name == 'c2dsr::' + n[len('c2dsr_'):]


def test_torch_op_refuses_host_tensors():
    import pytest
    torch.ops.load_library(EXT)
    x = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match='must be on the HIP device'):
        torch.ops.c2dsr.f32_to_bf16(x, 32, x)
