"""Flat, HBM-resident parameter store.

All trainable parameters of the model live in ONE contiguous fp32 buffer (16-B
aligned slices); their gradients in a second one ("fresh" = this step's gradient,
also the data-parallel all-reduce bucket) and the epoch-long accumulation that the
reference's once-per-epoch ``zero_grad`` implies (trainer.py:42, Q3) in a third.
AdamW's state (m, v, vmax) is flat too, so one kernel updates everything
(c2dsr_adamw) and one collective reduces everything.
"""
from __future__ import annotations

import torch


class FlatStore:
    """``align``: every slice starts at a multiple of ``align`` floats (4 = 16 B; data parallel uses 4·world
    so the reduction ranges of c2dsr_amd/dp.py split into equal float4-aligned parts per rank)."""

    def __init__(self, params: list[tuple[str, torch.nn.Parameter]], device, align: int = 4, direct: bool = False):
        """``direct``: no separate per-step buffer — ``fresh`` IS the epoch accumulation ``accum`` (one
        device: nothing is reduced, the backward accumulates into it and AdamW only reads it)."""
        self.align = align
        self.direct = direct
        seen = {}
        entries = []
        off = 0
        for name, p in params:
            if id(p) in seen:
                continue
            seen[id(p)] = name
            n = p.numel()
            entries.append((name, p, off, n))
            off += self.padded(n)
        self.numel = off
        self.device = device
        self.param = torch.zeros(off, device=device, dtype=torch.float32)
        self.accum = torch.zeros(off, device=device, dtype=torch.float32)
        self.fresh = self.accum if direct else torch.zeros(off, device=device, dtype=torch.float32)
        self.entries = entries
        self.names = [e[0] for e in entries]
        for name, p, o, n in entries:
            self.param[o:o + n].copy_(p.detach().reshape(-1).to(device))
            p.data = self.param[o:o + n].view(p.shape)
            p.grad = self.fresh[o:o + n].view(p.shape)

    def padded(self, n: int) -> int:
        return (n + self.align - 1) // self.align * self.align

    def params(self):
        return [p for _, p, _, _ in self.entries]

    def slices(self):
        return [(name, o, n) for name, _, o, n in self.entries]

    def reattach_grads(self):
        """Make every .grad a view of the fresh buffer again (after a user reset it)."""
        for _, p, o, n in self.entries:
            if p.grad is None or p.grad.data_ptr() != self.fresh[o:].data_ptr():
                if p.grad is not None:
                    self.fresh[o:o + n].add_(p.grad.reshape(-1))
                p.grad = self.fresh[o:o + n].view(p.shape)

    def release_accum(self):
        """ZeRO-1 keeps the epoch accumulation for this rank's shard only (optim.FlatAdamW): the full-size
        buffer is freed and grad_total is unavailable."""
        if self.direct:
            raise RuntimeError('the direct store has no separate accumulator')
        self.accum = None

    def grad_total(self, name):
        """Accumulated gradient (epoch accumulator + this step's) of one parameter."""
        if self.accum is None:
            raise RuntimeError('ZeRO-1: the accumulated gradient is sharded across ranks (FlatAdamW.accum holds '
                               'this rank\'s shard); grad_total is unavailable')
        for nm, p, o, n in self.entries:
            if nm == name:
                if self.direct:
                    return self.accum[o:o + n].view(p.shape)
                return (self.accum[o:o + n] + self.fresh[o:o + n]).view(p.shape)
        raise KeyError(name)
