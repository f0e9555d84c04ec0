"""Fused SGD(+momentum, weight decay, nesterov) and Adam/AdamW over flat
parameter groups — ``csrc/kernels/optim.hip``.

One kernel launch per group per step; the gradient average over data-parallel
ranks (``1/world``) and any loss scale are folded into ``grad_scale`` so no
separate scaling pass runs.  ``shard`` restricts the update to a slice of the
group — the parameter-server / ZeRO shard this rank owns (``parallel/ps.py``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ..parallel.flat import FlatGroup

P, L, I, F = _lib.P, _lib.L, _lib.I, _lib.F
_lib.register("kfa_sgd_step", [P, P, P, I, P, L, F, F, F, F, I, F, I, P])
_lib.register("kfa_adam_step", [P, P, P, I, P, P, L, F, F, F, F, F, F, F, F, P])
_lib.register("kfa_f32_to_bf16", [P, P, L, P])
_lib.register("kfa_sumsq", [P, I, L, P, P])


def _slice(t: Optional[torch.Tensor], rng: Optional[Tuple[int, int]]):
    if t is None or rng is None:
        return t
    return t[rng[0]:rng[1]]


class _FusedBase:
    def __init__(self, groups: Sequence[FlatGroup], lr: float, weight_decay: float,
                 decay_groups: Optional[Sequence[str]] = None):
        self.groups: List[FlatGroup] = list(groups)
        self.lr = lr
        self.weight_decay = weight_decay
        self.decay_groups = set(decay_groups) if decay_groups is not None else {"weights"}
        self.step_count = 0
        self.shards: Dict[int, Tuple[int, int]] = {}

    def set_shard(self, group_index: int, start: int, end: int) -> None:
        self.shards[group_index] = (start, end)

    def _wd(self, g: FlatGroup) -> float:
        return self.weight_decay if g.name in self.decay_groups or not g.name else 0.0

    def _cpu_check(self, g: FlatGroup) -> bool:
        return not g.data.is_cuda

    def sync_compute_copy(self) -> None:
        """Rewrite bf16 compute weights from the fp32 masters (after a broadcast / load)."""
        for g in self.groups:
            if g.master is not None:
                if g.data.is_cuda:
                    _lib.call("kfa_f32_to_bf16", _lib.ptr(g.master), _lib.ptr(g.data), g.numel, _lib.stream())
                else:
                    g.data.copy_(g.master)

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        out = torch.zeros(1, dtype=torch.float32, device=self.groups[0].device)
        for g in self.groups:
            if g.grad.is_cuda:
                _lib.call("kfa_sumsq", _lib.ptr(g.grad), int(g.grad.dtype == torch.bfloat16), g.numel,
                          _lib.ptr(out), _lib.stream())
            else:
                out += g.grad.float().pow(2).sum()
        return out.sqrt() * grad_scale


class FusedSGD(_FusedBase):
    def __init__(self, groups, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0, nesterov=False,
                 decay_groups=None):
        super().__init__(groups, lr, weight_decay, decay_groups)
        self.momentum = momentum
        self.dampening = dampening
        self.nesterov = nesterov
        self.mom = [torch.zeros(g.numel, dtype=torch.float32, device=g.device) if momentum else None
                    for g in self.groups]

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        lr = self.lr if lr is None else lr
        first = int(self.step_count == 0)
        for gi, g in enumerate(self.groups):
            rng = self.shards.get(gi)
            w = _slice(g.fp32, rng)
            wb = _slice(g.data, rng) if g.master is not None else None
            gr = _slice(g.grad, rng)
            mom = _slice(self.mom[gi], rng)
            n = w.numel()
            if n == 0:
                continue
            if self._cpu_check(g):
                d = gr.float() * grad_scale + self._wd(g) * w
                if mom is not None:
                    if first:
                        mom.copy_(d)
                    else:
                        mom.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                    d = d + self.momentum * mom if self.nesterov else mom
                w.add_(d, alpha=-lr)
                if wb is not None:
                    wb.copy_(w)
                continue
            _lib.call("kfa_sgd_step", _lib.ptr(w), _lib.ptr(wb), _lib.ptr(gr), int(gr.dtype == torch.bfloat16),
                      _lib.ptr(mom), n, lr, self.momentum, self.dampening, self._wd(g), int(self.nesterov),
                      grad_scale, first, _lib.stream())
        self.step_count += 1


class FusedAdam(_FusedBase):
    def __init__(self, groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decay_groups=None):
        super().__init__(groups, lr, weight_decay, decay_groups)
        self.b1, self.b2 = betas
        self.eps = eps
        self.m = [torch.zeros(g.numel, dtype=torch.float32, device=g.device) for g in self.groups]
        self.v = [torch.zeros(g.numel, dtype=torch.float32, device=g.device) for g in self.groups]

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        lr = self.lr if lr is None else lr
        self.step_count += 1
        t = self.step_count
        bc1 = 1.0 - self.b1 ** t
        bc2 = 1.0 - self.b2 ** t
        for gi, g in enumerate(self.groups):
            rng = self.shards.get(gi)
            w = _slice(g.fp32, rng)
            wb = _slice(g.data, rng) if g.master is not None else None
            gr = _slice(g.grad, rng)
            m, v = _slice(self.m[gi], rng), _slice(self.v[gi], rng)
            n = w.numel()
            if n == 0:
                continue
            wd = self._wd(g)
            if self._cpu_check(g):
                d = gr.float() * grad_scale
                m.mul_(self.b1).add_(d, alpha=1 - self.b1)
                v.mul_(self.b2).addcmul_(d, d, value=1 - self.b2)
                denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
                w.mul_(1 - lr * wd).addcdiv_(m, denom, value=-lr / bc1)
                if wb is not None:
                    wb.copy_(w)
                continue
            _lib.call("kfa_adam_step", _lib.ptr(w), _lib.ptr(wb), _lib.ptr(gr), int(gr.dtype == torch.bfloat16),
                      _lib.ptr(m), _lib.ptr(v), n, lr, self.b1, self.b2, self.eps, wd, bc1, bc2, grad_scale,
                      _lib.stream())
