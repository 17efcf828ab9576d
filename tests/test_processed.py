"""f2: the reference's processed on-disk formats (dataloader.py:24-35, utils/graph.py:99-107).

The fixtures under tests/golden/processed_<cfg>/ are the very {train,val,test}.pkl and graph.pkl the
reference wrote when driven with --use_raw --save_processed (tools/gen_fixtures.py --traj).  The
use_raw=False path must read them (through the restricted unpickler) into exactly the lists and CSR
the raw path produces, and must refuse any pickle that names code."""
import os
import pickle
import random
import shutil
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from c2dsr_amd import dataloader as DL
from c2dsr_amd import graph as GR
from c2dsr_amd import processed
from tests import goldens as G


def _args(path_raw, path_data, use_raw, name='base'):
    c = G.CONFIGS[name]
    return SimpleNamespace(path_raw=str(path_raw), path_data=str(path_data), use_raw=use_raw, save_processed=True,
                           len_max=c['len_max'], n_neg_sample=G.N_NEG, batch_size=G.BATCH, batch_size_eval=64,
                           num_workers=0)


def _fields(rows, k):
    return DL.to_arrays(rows)[:k]


@pytest.mark.parametrize('name', ['base', 'var'])
def test_reference_processed_lists_read_bit_exact(name):
    d = G.load(f'data_{name}.npz')
    src = os.path.join(G.GOLDEN, f'processed_{name}')
    args = _args('/nonexistent', src, False, name)
    tr, va, te = DL.get_dataloader(args)
    assert (args.n_item_a, args.n_item_b) == (G.CONFIGS[name]['n_a'], G.CONFIGS[name]['n_b'])
    for mode, ds, k in (('train', tr.dataset, 14), ('val', va.dataset, 11), ('test', te.dataset, 11)):
        assert len(ds) == int(d[f'n_{mode}'])
        for j, col in enumerate(_fields(ds.data, k)):
            np.testing.assert_array_equal(col, d[f'{mode}_{j}'], err_msg=f'{mode} field {j}')


@pytest.mark.parametrize('name', ['base'])
def test_reference_processed_graph_read_bit_exact(name):
    g = G.load(f'graph_{name}.npz')
    c = G.CONFIGS[name]
    args = _args('/nonexistent', os.path.join(G.GOLDEN, f'processed_{name}'), False, name)
    args.n_item_a, args.n_item_b = c['n_a'], c['n_b']
    args.n_item = c['n_a'] + c['n_b'] + 1
    gs, gp = GR.make_graph(args, '/nonexistent/train_new.txt')
    for k, csr in (('share', gs), ('specific', gp)):
        r, col, v = csr.coo()  # the reference's COO is uncoalesced; compare the triples as sets
        ref = sorted(zip(g[f'{k}_row'].tolist(), g[f'{k}_col'].tolist(), g[f'{k}_val'].view(np.uint32).tolist()))
        assert sorted(zip(r.tolist(), col.tolist(), v.view(np.uint32).tolist())) == ref, k


def test_raw_path_writes_what_the_processed_path_reads(tmp_path):
    """use_raw=True processes the raw files and saves {mode}.pkl / graph.pkl (dataloader.py:26-29,
    utils/graph.py:101-103); a second run with use_raw=False reads them back unchanged."""
    d = G.load('data_base.npz')
    raw, data = tmp_path / 'raw', tmp_path / 'data'
    raw.mkdir()
    for mode in ('train', 'val', 'test'):
        (raw / f'{mode}_new.txt').write_bytes(d[f'raw_{mode}'].tobytes())
    for f in ('items_a.txt', 'items_b.txt'):
        shutil.copy(os.path.join(G.GOLDEN, 'processed_base', f), raw / f)
    random.seed(3407)
    a1 = _args(raw, data, True)
    l1 = DL.get_dataloader(a1)
    g1 = GR.make_graph(a1, str(raw / 'train_new.txt'))
    for f in ('items_a.txt', 'items_b.txt'):
        shutil.copy(raw / f, data / f)
    a2 = _args(tmp_path / 'gone', data, False)
    l2 = DL.get_dataloader(a2)
    g2 = GR.make_graph(a2, '/nonexistent')
    for x, y in zip(l1, l2):
        assert x.dataset.data == y.dataset.data
    for x, y in zip(g1, g2):
        np.testing.assert_array_equal(x.rowptr, y.rowptr)
        np.testing.assert_array_equal(x.col, y.col)
        np.testing.assert_array_equal(x.val, y.val)
    for j in range(14):  # and they are the reference's lists
        np.testing.assert_array_equal(DL.to_arrays(l2[0].dataset.data)[j], d[f'train_{j}'])


class _Evil:
    def __reduce__(self):
        return (os.system, ('true',))


def test_processed_reader_refuses_code(tmp_path):
    p = tmp_path / 'train.pkl'
    p.write_bytes(pickle.dumps([[1, 2, 3], _Evil()]))
    with pytest.raises(pickle.UnpicklingError):
        processed.load_lists(str(p))
    q = tmp_path / 'graph.pkl'
    q.write_bytes(pickle.dumps((torch.zeros(2).to_sparse(), _Evil())))
    with pytest.raises(pickle.UnpicklingError):
        processed.load_graph(str(q))


def test_missing_inputs_name_the_file(tmp_path):
    with pytest.raises(FileNotFoundError, match='train.pkl'):
        processed.load_lists(str(tmp_path / 'train.pkl'))
    a = _args(tmp_path, tmp_path, True)
    a.n_item_a, a.n_item_b = 3, 4
    with pytest.raises(FileNotFoundError, match='train_new.txt'):
        DL.CDSRDataset(a, 'train')
