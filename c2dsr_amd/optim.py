"""AdamW(amsgrad) over the flat parameter store — the reference's optimizer
(trainer.py:21-22: torch.optim.AdamW(lr, weight_decay=l2, amsgrad=True)) as one
fused HIP kernel per step, keeping torch.optim.Optimizer's surface (param_groups,
state_dict, zero_grad) so StepLR and main.py work unchanged (main.py:103,115,140-142).
"""
from __future__ import annotations

import torch

from ._lib import stage_ops
from .flat import FlatStore


class FlatAdamW(torch.optim.Optimizer):
    """``zero``: a c2dsr_amd.dp.Zero1 — ZeRO-1: the summed gradient of this rank's parts
    arrives reduce-scattered in ``zero.gshard``; m / v / vmax and the epoch accumulation are kept for the
    shard only, the kernel runs once per owned part, and the updated parts are all-gathered."""

    def __init__(self, flat: FlatStore, lr=1e-3, weight_decay=5e-4, betas=(0.9, 0.999), eps=1e-8, amsgrad=True,
                 zero=None):
        if not amsgrad:
            raise ValueError('the C2DSR path uses amsgrad=True (trainer.py:21-22)')
        super().__init__(flat.params(), dict(lr=lr, weight_decay=weight_decay, betas=betas, eps=eps, amsgrad=True))
        self.flat = flat
        self.zero = zero
        dev = flat.device
        n = flat.numel if zero is None else zero.shard_numel
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.vmax = torch.zeros(n, device=dev)
        if zero is None:
            self.accum = flat.accum
        else:
            self.accum = torch.zeros(n, device=dev)
            flat.release_accum()  # the shard above replaces it (1/p of the state, not 1 + 1/p)
        self.n_steps = 0
        self.accumulate = True  # grads accumulate until zero_grad (Q3)
        # data parallel: the step's reduction ranges with their collectives' handles in issue order
        # (DPComm.in_order); the next step() waits for each range's sum just before updating that range, so the
        # update of the early ranges runs while the last ones are still being summed
        self.comm = None

    def sync_grads(self):
        """Data parallel: make the current stream wait for every pending range's sum (the gradient store is then
        final) — for a caller that reads the gradients between the backward and step()."""
        for _, _, w in self.comm or ():
            w.wait()

    def zero_grad(self, set_to_none: bool = True):
        """Reference semantics: clears the epoch accumulation (grads would be None)."""
        self.accum.zero_()
        self.flat.fresh.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        g = self.param_groups[0]
        self.n_steps += 1
        b1, b2 = g['betas']
        f = self.flat
        hyper = (float(g['lr']), float(g['weight_decay']), float(b1), float(b2), float(g['eps']), self.n_steps)
        comm, self.comm = self.comm, None
        acc = self.accum if self.accumulate else None
        if self.zero is None and comm is None:
            # direct store (one device): fresh is accum — read only, 36 B/param; without epoch accumulation
            # the same buffer is this step's gradient and is cleared
            stage_ops().adamw_step(f.param, f.fresh, acc, self.m, self.v, self.vmax, *hyper)
        elif self.zero is None:  # range by range as the sums land (the update is elementwise: the same bits)
            for lo, hi, w in comm:
                w.wait()
                stage_ops().adamw_step(f.param[lo:hi], f.fresh[lo:hi], None if acc is None else acc[lo:hi],
                                       self.m[lo:hi], self.v[lo:hi], self.vmax[lo:hi], *hyper)
        else:
            z = self.zero
            order = [(lo, hi, None) for lo, hi, _, _, _ in z.parts] if comm is None else comm
            part = {(lo, hi): (olo, ohi, off) for lo, hi, olo, ohi, off in z.parts}
            for lo, hi, w in order:
                if w is not None:
                    w.wait()
                olo, ohi, off = part[(lo, hi)]
                sl = slice(off, off + ohi - olo)
                stage_ops().adamw_step(f.param[olo:ohi], z.gshard[sl], None if acc is None else acc[sl],
                                       self.m[sl], self.v[sl], self.vmax[sl], *hyper)
            f.fresh.zero_()  # the next backward accumulates into it
            for w in z.gather():
                w.wait()
        from .ops import WEIGHTS
        WEIGHTS.bump()  # the weights' bf16 images are stale now
        return None
