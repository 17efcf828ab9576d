"""Host logic of the classifier head's sweep plans (c2dsr_amd/losshead.py): the fwd column splits (split_count) and the
dW sweep's plan (dw_plan over row splits, stream-K and whole rounds + a split remainder), on a 256-CU device.  The
GPU tests check what each plan computes (tests/test_gpu_ce3.py: every form against float64); these pin which form
is chosen at the benchmarked shapes and that a plan is always one the kernels accept."""
import pytest

from c2dsr_amd import losshead as L


@pytest.fixture(autouse=True)
def _cus(monkeypatch):
    monkeypatch.setattr(L, '_ncu', lambda: 256)


@pytest.mark.parametrize('n,Mv,x3,expect', [
    (63937, 18944, True, 1),     # MB head b: 500 row blocks = 1.95 rounds, one split added onto the gradient
    (36845, 18944, True, -8),    # MB head a: 288 row blocks = 256 unsplit + 32 split 8 ways
    (36845, 18944, False, -8),
    (63937, 18944, False, 1),
    (29207, 9472, False, 1),     # FK head a: 229 row blocks, one round
])
def test_dw_plan_at_benchmarked_shapes(n, Mv, x3, expect):
    assert L.dw_plan(n, Mv, x3, 256) == expect


@pytest.mark.parametrize('n', [31, 700, 4099, 32768, 32769, 36845, 40000, 63937, 100000, 300000])
@pytest.mark.parametrize('Mv', [33, 1000, 9472, 18944])
@pytest.mark.parametrize('x3', [True, False])
def test_dw_plan_is_valid(n, Mv, x3):
    p = L.dw_plan(n, Mv, x3, 256)
    assert -64 <= p <= 64  # ce_head_backward's n_rsplit range
    blocks = -(-n // 128)
    if p < 0:  # the remainder form needs whole rounds and a remainder
        assert blocks > 256 and blocks % 256 != 0 and p <= -2
    # without both gradients only row splits are possible (stream-K and the remainder form add onto gW / gb)
    assert L.dw_plan(n, Mv, x3, 256, both_grads=False) >= 1


def test_dw_split_count_least_cost_smallest_on_ties():
    split, _ = L._dw_costs(34886, 9472, False)
    k = L.dw_split_count(34886, 9472, False)
    assert split[k] == min(split.values())
    assert all(split[s] > split[k] + 1e-9 for s in split if s < k)


def test_dw_plan_other_widths_keep_split_count():
    assert L.dw_plan(4099, 777, True, 128) == L.split_count(4099, 128)


def test_fwd_split_count_whole_rounds():
    # 148 row blocks (MB head, Mv = 18,944): 12 splits = 1776 workgroups, 6.94 rounds of 256
    assert L.split_count(18944, 128) == 12
    assert L.split_count(64, 128) >= 1


def test_fwd_split_count_fitted():
    # fp32 mode at the MB heads (Mv = 18,944): head a 5 splits (fewer U slabs at equal sweep time), head b 12
    assert L.fwd_split_count(18944, 36845, True) == 5
    assert L.fwd_split_count(18944, 63937, True) == 12
    # bf16 (64-row tiles): 5 at the MB heads, 3 at the Food-Kitchen heads; other widths keep split_count
    assert L.fwd_split_count(18944, 36845, False) == 5 and L.fwd_split_count(18944, 63937, False) == 5
    assert L.fwd_split_count(9472, 34886, False) == 3
    assert L.fwd_split_count(18944, 36845, True, d=128) == L.split_count(18944, 128)
    for Mv in (1, 64, 9472, 40960):
        for n in (31, 36845, 63937):
            assert 1 <= L.fwd_split_count(Mv, n, True) <= 16
