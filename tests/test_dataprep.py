"""a1/a2 bit-exactness: index/mask construction and graph CSR vs the reference's
own outputs (golden fixtures made by tools/gen_fixtures.py)."""
import hashlib
import os
import random

import numpy as np
import pytest

from c2dsr_amd import dataloader as DL
from c2dsr_amd import graph as GR
from tests import goldens as G


def _write_raw(tmp_path, name):
    d = G.load(f'data_{name}.npz')
    for mode in ('train', 'val', 'test'):
        (tmp_path / f'{mode}_new.txt').write_bytes(d[f'raw_{mode}'].tobytes())
    return d


@pytest.mark.parametrize('name', ['base'])
def test_preprocess_lists_bit_exact(tmp_path, name):
    d = _write_raw(tmp_path, name)
    c = G.CONFIGS[name]
    random.seed(3407)  # main.py:91, before the three CDSRDataset constructions
    tr = DL.preprocess_train(GR.read_sequences(str(tmp_path / 'train_new.txt')), c['n_a'], c['n_b'], c['len_max'])
    va = DL.preprocess_evaluate(GR.read_sequences(str(tmp_path / 'val_new.txt')), c['n_a'], c['n_b'], c['len_max'],
                                G.N_NEG)
    te = DL.preprocess_evaluate(GR.read_sequences(str(tmp_path / 'test_new.txt')), c['n_a'], c['n_b'], c['len_max'],
                                G.N_NEG)
    for mode, rows, k in (('train', tr, 14), ('val', va, 11), ('test', te, 11)):
        assert len(rows) == int(d[f'n_{mode}'])
        arr = DL.to_arrays(rows)
        for j in range(k):
            np.testing.assert_array_equal(arr[j], d[f'{mode}_{j}'], err_msg=f'{mode} field {j}')


@pytest.mark.parametrize('name', ['base'])
def test_graph_csr_bit_exact(tmp_path, name):
    _write_raw(tmp_path, name)
    c = G.CONFIGS[name]
    n = c['n_a'] + c['n_b'] + 1
    gs, gp = GR.preprocess_graph(str(tmp_path / 'train_new.txt'), c['n_a'], n)
    g = G.load(f'graph_{name}.npz')
    for key, ours in (('share', gs), ('specific', gp)):
        r, cc, v = ours.coo()
        ref = sorted(zip(g[f'{key}_row'].tolist(), g[f'{key}_col'].tolist(), g[f'{key}_val'].view(np.uint32).tolist()))
        got = sorted(zip(r.tolist(), cc.tolist(), v.view(np.uint32).tolist()))
        assert got == ref, key
        # transpose holds the same triples
        t = ours.transpose()
        rt, ct, vt = t.coo()
        assert sorted(zip(ct.tolist(), rt.tolist(), vt.view(np.uint32).tolist())) == ref


FK_RAW = '/root/reference/data/raw/Food-Kitchen/val_new.txt'


@pytest.mark.skipif(not os.path.exists(FK_RAW), reason='Food-Kitchen raw file only in the build container')
def test_food_kitchen_standin_bit_exact():
    """The real FK val file processed as train/eval data and as the graph source."""
    fk = G.load('fk_data.npz')
    seqs = GR.read_sequences(FK_RAW)
    n_a, n_b = 29207, 34886
    random.seed(3407)
    tr = np.asarray(DL.preprocess_train(seqs, n_a, n_b, 15), dtype=np.int64)
    assert list(tr.shape) == fk['trainlike_shape'].tolist()
    np.testing.assert_array_equal(tr[:64], fk['trainlike_head'])
    assert hashlib.sha256(tr.tobytes()).digest() == fk['trainlike_sha256'].tobytes()
    ev = DL.preprocess_evaluate(seqs, n_a, n_b, 15, 999)
    flat = np.concatenate([np.concatenate([np.asarray(x, dtype=np.int64) for x in r]) for r in ev])
    assert hashlib.sha256(flat.tobytes()).digest() == fk['evallike_sha256'].tobytes()
    gs, gp = GR.preprocess_graph(seqs, n_a, n_a + n_b + 1)
    assert gs.nnz == int(fk['share_nnz']) and gp.nnz == int(fk['specific_nnz'])
