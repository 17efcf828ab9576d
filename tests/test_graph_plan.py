"""CPU checks of the SpMM load-balancing plan (c2dsr_amd/graph.py:work_plan)."""
import numpy as np

from c2dsr_amd.graph import normalized_csr, work_plan


def test_work_plan_covers_every_edge_once():
    rng = np.random.default_rng(0)
    n = 300
    edges = np.concatenate([rng.integers(0, n, (4000, 2)), np.stack([np.full(1000, 7), rng.integers(0, n, 1000)], 1)])
    g = normalized_csr(edges, n)
    work, split, nslot = work_plan(g, split=64)
    cover = np.zeros(g.nnz, dtype=int)
    for row, eb, ee, slot in work:
        assert g.rowptr[row] <= eb <= ee <= g.rowptr[row + 1]
        assert ee - eb <= 64
        cover[eb:ee] += 1
    assert (cover == 1).all()
    rows_in_work = set(work[:, 0].tolist())
    assert rows_in_work == set(range(n))
    assert split.shape[0] >= 1 and 7 in split[:, 0]
    slots = work[work[:, 3] >= 0, 3]
    assert sorted(slots.tolist()) == list(range(nslot))
    for row, sb, se, _ in split:
        pieces = work[work[:, 0] == row]
        assert (pieces[:, 3] == np.arange(sb, se)).all()


def test_flat_generator_edges_match_reference_rules():
    """The vectorised C5 generator's edges equal graph.transition_edges (the reference's rules) on
    the same sequences."""
    import numpy as np
    from c2dsr_amd import graph as GR
    from c2dsr_amd import synth
    items, off = synth.make_flat_sequences(500, 300, 400, 30, seed=4)
    assert off[-1] == items.size and items.min() >= 0 and items.max() < 700
    seqs = [items[off[i]:off[i + 1]].tolist() for i in range(500)]
    sh_ref, sp_ref = GR.transition_edges(seqs, 300)
    sh, sp = synth.transition_edges_flat(items, off, 300)
    np.testing.assert_array_equal(sh, sh_ref)
    np.testing.assert_array_equal(sp, sp_ref)
