"""Loading helpers for the golden fixtures made by tools/gen_fixtures.py."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

# must match tools/gen_fixtures.py CONFIGS
CONFIGS = {
    'base': dict(n_a=40, n_b=60, len_max=8, len_rec=4, d_latent=16,
                 n_gnn=1, n_attn=1, n_head=1, norm_first=False, d_bias=False, shared_item_embed=False),
    'var': dict(n_a=40, n_b=60, len_max=8, len_rec=4, d_latent=16,
                n_gnn=2, n_attn=2, n_head=2, norm_first=True, d_bias=True, shared_item_embed=False),
    'shared': dict(n_a=40, n_b=60, len_max=8, len_rec=4, d_latent=16,
                   n_gnn=1, n_attn=1, n_head=1, norm_first=False, d_bias=False, shared_item_embed=True),
}
N_NEG = 10
BATCH = 16


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def oracle_cfg(name, dropout_gnn=0.0, dropout_attn=0.0):
    c = CONFIGS[name]
    return dict(d_latent=c['d_latent'], n_item_a=c['n_a'], n_item_b=c['n_b'], idx_pad=c['n_a'] + c['n_b'],
                len_rec=c['len_rec'], lambda_loss=0.7, n_gnn=c['n_gnn'], n_attn=c['n_attn'], n_head=c['n_head'],
                norm_first=c['norm_first'], d_bias=c['d_bias'], shared_item_embed=c['shared_item_embed'],
                dropout_gnn=dropout_gnn, dropout_attn=dropout_attn)


def init_params(name):
    m = load(f'model_{name}.npz')
    return {k[len('init/'):]: torch.from_numpy(m[k].copy()) for k in m.files if k.startswith('init/')
            and not k.endswith('attn_mask')}


def graphs_coo(name):
    g = load(f'graph_{name}.npz')
    out = {}
    for k in ('share', 'specific'):
        out[k] = (torch.from_numpy(g[f'{k}_row']), torch.from_numpy(g[f'{k}_col']), torch.from_numpy(g[f'{k}_val']))
    return out


def train_rows(name):
    d = load(f'data_{name}.npz')
    return [d[f'train_{j}'] for j in range(14)]


def batch(name, lo, n):
    rows = train_rows(name)
    return tuple(torch.from_numpy(r[lo:lo + n].copy()) for r in rows)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
