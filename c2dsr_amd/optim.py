"""AdamW(amsgrad) over the flat parameter store — the reference's optimizer
(trainer.py:21-22: torch.optim.AdamW(lr, weight_decay=l2, amsgrad=True)) as one
fused HIP kernel per step, keeping torch.optim.Optimizer's surface (param_groups,
state_dict, zero_grad) so StepLR and main.py work unchanged (main.py:103,115,140-142).
"""
from __future__ import annotations

import torch

from ._lib import lib, stream
from .flat import FlatStore


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, flat: FlatStore, lr=1e-3, weight_decay=5e-4, betas=(0.9, 0.999), eps=1e-8, amsgrad=True):
        if not amsgrad:
            raise ValueError('the C2DSR path uses amsgrad=True (trainer.py:21-22)')
        super().__init__(flat.params(), dict(lr=lr, weight_decay=weight_decay, betas=betas, eps=eps, amsgrad=True))
        self.flat = flat
        dev = flat.device
        self.m = torch.zeros(flat.numel, device=dev)
        self.v = torch.zeros(flat.numel, device=dev)
        self.vmax = torch.zeros(flat.numel, device=dev)
        self.n_steps = 0
        self.accumulate = True  # grads accumulate until zero_grad (Q3)

    def zero_grad(self, set_to_none: bool = True):
        """Reference semantics: clears the epoch accumulation (grads would be None)."""
        self.flat.accum.zero_()
        self.flat.fresh.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        g = self.param_groups[0]
        self.n_steps += 1
        b1, b2 = g['betas']
        f = self.flat
        lib('c2dsr_adamw', f.param, f.fresh, f.accum if self.accumulate else None, self.m, self.v, self.vmax, f.numel,
            float(g['lr']), float(g['weight_decay']), float(b1), float(b2), float(g['eps']), self.n_steps, stream())
        from .ops import WEIGHTS
        WEIGHTS.bump()  # the weights' bf16 images are stale now
        return None
