"""Flat fp32 arenas for parameters, gradients and optimizer state.

Every parameter (and its .grad) becomes a view into ONE contiguous buffer,
each slot padded to 64 elements (256 B), so that
  * the fused SGD kernel updates all 20.7M parameters in one launch,
  * gradient buckets are contiguous slices (no copy-in/copy-out around the
    RCCL all-reduce, like DDP's gradient_as_bucket_view),
  * init-time parameter sync is ONE broadcast.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

ALIGN = 64


class FlatArena:
    def __init__(self, params: List[torch.nn.Parameter], device, with_grads: bool = True, order=None):
        """``order``: parameter indices in the sequence their slots are laid out
        (gradient-ready order, so reducer buckets are contiguous)."""
        self.params = params
        self.order = list(order) if order is not None else list(range(len(params)))
        if sorted(self.order) != list(range(len(params))):
            raise ValueError("order must be a permutation of the parameter indices")
        self.offsets: List[Tuple[int, int]] = [(0, 0)] * len(params)
        off = 0
        for i in self.order:
            n = params[i].numel()
            self.offsets[i] = (off, n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        dev = torch.device(device)
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev) if with_grads else None
        with torch.no_grad():
            for p, (o, n) in zip(params, self.offsets):
                self.data[o:o + n].copy_(p.detach().reshape(-1).to(device=dev, dtype=torch.float32))
                p.data = self.data[o:o + n].view_as(p)
        if with_grads:
            self.attach_grads()

    def attach_grads(self):
        for p, (o, n) in zip(self.params, self.offsets):
            p.grad = self.grad[o:o + n].view_as(p)

    def grad_views(self) -> List[torch.Tensor]:
        return [self.grad[o:o + n].view_as(p) for p, (o, n) in zip(self.params, self.offsets)]

    def slot(self, i: int) -> Tuple[int, int]:
        """(start, padded end) of parameter i in the arena."""
        o, n = self.offsets[i]
        return o, o + (n + ALIGN - 1) // ALIGN * ALIGN
