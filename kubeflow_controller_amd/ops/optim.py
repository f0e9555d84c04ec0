"""Fused SGD(+momentum, weight decay, nesterov) and Adam/AdamW over flat
parameter groups — ``csrc/kernels/optim.hip``.

One kernel launch per optimizer space per step; the gradient average over
data-parallel ranks (``1/world``) and any loss scale are folded into
``grad_scale`` so no separate scaling pass runs.  A space is a whole flat group
or the compact parameter-server / ZeRO shard a rank owns (``parallel/ps.py``):
the optimizer state is allocated at the space's size, so an owner holds state
only for what it owns.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ..parallel.flat import FlatGroup

P, L, I, F = _lib.P, _lib.L, _lib.I, _lib.F
_lib.register("kfa_sgd_step", [P, P, P, I, P, L, F, F, F, F, I, F, I, P])
_lib.register("kfa_adam_step", [P, P, P, I, P, P, L, F, F, F, F, F, F, F, F, P, P])
_lib.register("kfa_adam_bc", [P, P, F, F, P])
_lib.register("kfa_adam_bc_seed", [P, P, F, F, I, P])
_lib.register("kfa_f32_to_bf16", [P, P, L, P])
_lib.register("kfa_sumsq", [P, I, L, P, P])


class OptSpace:
    """One contiguous region a fused optimizer updates in ONE launch: fp32
    weights ``w`` (updated in place), an optional low-precision compute copy
    ``wb`` rewritten from ``w`` in the same kernel, and the gradient ``grad``
    (bf16 or fp32).  A whole flat group (data-parallel all-reduce) or one
    rank's compact shard of it (parameter-server / ZeRO owner, ``parallel/ps.py``)."""

    __slots__ = ("name", "w", "wb", "_grad")

    def __init__(self, name: str, w: torch.Tensor, wb: Optional[torch.Tensor], grad):
        self.name = name
        self.w = w
        self.wb = wb
        self._grad = grad

    @classmethod
    def of_group(cls, g: FlatGroup) -> "OptSpace":
        return cls(g.name, g.fp32, g.data if g.master is not None else None, lambda: g.opt_grad)

    @property
    def grad(self) -> torch.Tensor:
        return self._grad() if callable(self._grad) else self._grad

    @property
    def numel(self) -> int:
        return self.w.numel()

    @property
    def device(self) -> torch.device:
        return self.w.device


def _as_spaces(items) -> List[OptSpace]:
    return [x if isinstance(x, OptSpace) else OptSpace.of_group(x) for x in items]


class _FusedBase:
    def __init__(self, spaces: Sequence, lr: float, weight_decay: float,
                 decay_groups: Optional[Sequence[str]] = None):
        self.spaces: List[OptSpace] = _as_spaces(spaces)
        self.lr = lr
        self.weight_decay = weight_decay
        self.decay_groups = set(decay_groups) if decay_groups is not None else {"weights"}
        self.step_count = 0

    def _wd(self, s: OptSpace) -> float:
        return self.weight_decay if s.name in self.decay_groups or not s.name else 0.0

    @staticmethod
    def _cpu(s: OptSpace) -> bool:
        return not s.w.is_cuda

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        """L2 norm of the gradient this rank holds (its shard in the sharded layouts)."""
        out = torch.zeros(1, dtype=torch.float32, device=self.spaces[0].device)
        for s in self.spaces:
            g = s.grad
            if g.numel() == 0:
                continue
            if g.is_cuda:
                _lib.call("kfa_sumsq", _lib.ptr(g), int(g.dtype == torch.bfloat16), g.numel(),
                          _lib.ptr(out), _lib.stream())
            else:
                out += g.float().pow(2).sum()
        return out.sqrt() * grad_scale


class FusedSGD(_FusedBase):
    def __init__(self, groups, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=0.0, nesterov=False,
                 decay_groups=None):
        super().__init__(groups, lr, weight_decay, decay_groups)
        self.momentum = momentum
        self.dampening = dampening
        self.nesterov = nesterov
        self.mom = [torch.zeros(s.numel, dtype=torch.float32, device=s.device) if momentum else None
                    for s in self.spaces]
        self._first = 1  # set per step by begin_step

    def begin_step(self) -> None:
        """Open one optimizer step whose updates are issued per range (``update``)."""
        self._first = int(self.step_count == 0)
        self.step_count += 1

    @torch.no_grad()
    def update(self, si: int, a: int, b: int, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        """Elements [a, b) of space ``si`` in the step opened by ``begin_step`` (the
        update is elementwise, so any cut of a space into ranges gives the whole-space result)."""
        if b <= a:
            return
        lr = self.lr if lr is None else lr
        s, mom = self.spaces[si], self.mom[si]
        w, wb, gr = s.w[a:b], (s.wb[a:b] if s.wb is not None else None), s.grad[a:b]
        mom = mom[a:b] if mom is not None else None
        if self._cpu(s):
            d = gr.float() * grad_scale + self._wd(s) * w
            if mom is not None:
                if self._first:
                    mom.copy_(d)
                else:
                    mom.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                d = d + self.momentum * mom if self.nesterov else mom
            w.add_(d, alpha=-lr)
            if wb is not None:
                wb.copy_(w)
            return
        _lib.call("kfa_sgd_step", _lib.ptr(w), _lib.ptr(wb), _lib.ptr(gr), int(gr.dtype == torch.bfloat16),
                  _lib.ptr(mom), b - a, lr, self.momentum, self.dampening, self._wd(s), int(self.nesterov),
                  grad_scale, self._first, _lib.stream())

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        self.begin_step()
        for si, s in enumerate(self.spaces):
            self.update(si, 0, s.numel, grad_scale, lr)


class FusedAdam(_FusedBase):
    def __init__(self, groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decay_groups=None):
        super().__init__(groups, lr, weight_decay, decay_groups)
        self.b1, self.b2 = betas
        self.eps = eps
        self.m = [torch.zeros(s.numel, dtype=torch.float32, device=s.device) for s in self.spaces]
        self.v = [torch.zeros(s.numel, dtype=torch.float32, device=s.device) for s in self.spaces]
        # GPU: the step count t and (1 - b1^t, 1 - b2^t) live on the device, advanced
        # by kfa_adam_bc inside the step, so the step replays from a HIP graph
        dev = self.spaces[0].device if self.spaces else torch.device("cpu")
        self._t = torch.zeros(1, dtype=torch.int32, device=dev) if dev.type == "cuda" else None
        self._bc = torch.ones(2, dtype=torch.float32, device=dev) if dev.type == "cuda" else None

    def begin_step(self) -> None:
        """Open one optimizer step whose updates are issued per range (``update``):
        the step count and the bias corrections advance once, here."""
        if self._t is not None:
            # eager steps (and resumes) re-seed the device count inside the same launch; a
            # captured step advances it on the device (graph replay)
            seed = -1 if torch.cuda.is_current_stream_capturing() else self.step_count
            _lib.call("kfa_adam_bc_seed", _lib.ptr(self._t), _lib.ptr(self._bc), self.b1, self.b2, seed,
                      _lib.stream())
        self.step_count += 1

    @torch.no_grad()
    def update(self, si: int, a: int, b: int, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        """Elements [a, b) of space ``si`` in the step opened by ``begin_step`` (elementwise:
        any cut of a space into ranges gives the whole-space result bit for bit)."""
        if b <= a:
            return
        lr = self.lr if lr is None else lr
        t = self.step_count
        bc1 = 1.0 - self.b1 ** t
        bc2 = 1.0 - self.b2 ** t
        s = self.spaces[si]
        w, wb, gr = s.w[a:b], (s.wb[a:b] if s.wb is not None else None), s.grad[a:b]
        m, v = self.m[si][a:b], self.v[si][a:b]
        wd = self._wd(s)
        if self._cpu(s):
            d = gr.float() * grad_scale
            m.mul_(self.b1).add_(d, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(d, d, value=1 - self.b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            w.mul_(1 - lr * wd).addcdiv_(m, denom, value=-lr / bc1)
            if wb is not None:
                wb.copy_(w)
            return
        _lib.call("kfa_adam_step", _lib.ptr(w), _lib.ptr(wb), _lib.ptr(gr), int(gr.dtype == torch.bfloat16),
                  _lib.ptr(m), _lib.ptr(v), b - a, lr, self.b1, self.b2, self.eps, wd, bc1, bc2, grad_scale,
                  _lib.ptr(self._bc), _lib.stream())

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, lr: Optional[float] = None) -> None:
        self.begin_step()
        for si, s in enumerate(self.spaces):
            self.update(si, 0, s.numel, grad_scale, lr)
