"""Flat parameter / gradient storage.

Every trainable tensor of one dtype group becomes a view into ONE contiguous
buffer (offsets padded to 8 elements = 16 B for bf16 / 32 B for fp32, total
padded to ``pad_to`` elements so it splits evenly into reduce-scatter shards).
The same layout is used for the gradient buffer, so:

* the fused optimizer (``ops/optim.py``) updates a whole group in ONE launch;
* data-parallel buckets are plain slices of the gradient buffer — RCCL
  all-reduces / reduce-scatters them without any pack/unpack copy;
* a bf16 group carries an fp32 master copy (mixed precision, SURVEY §2.6:
  "bf16 with fp32 master weights").
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

ALIGN = 8

# Direct-gradient protocol: a HIP backward kernel may write (+=) a parameter's
# gradient straight into its flat-buffer view and return ``None`` to autograd,
# skipping the AccumulateGrad add kernel; it then calls ``notify_grad_ready``
# so data-parallel bucket bookkeeping still sees the tensor as ready.
_READY_CB = {}


def direct_grad_view(p) -> Optional[torch.Tensor]:
    """The flat gradient view of ``p`` if it lives in a FlatGroup, else None."""
    if getattr(p, "_kfa_flat", False) and p.grad is not None:
        return p.grad
    return None


def set_ready_callback(p, cb) -> None:
    _READY_CB[id(p)] = cb


def notify_grad_ready(p) -> None:
    p._kfa_direct = True  # this backward delivered p's gradient directly (see register_ready_hook)
    cb = _READY_CB.get(id(p))
    if cb is not None:
        cb(p)


def register_ready_hook(p, hook):
    """Call ``hook(p)`` once per gradient contribution to ``p`` in a backward, by
    whichever route it arrives: a HIP backward that wrote the flat gradient and
    called :func:`notify_grad_ready`, or autograd's AccumulateGrad.  AccumulateGrad's
    post hook ALSO runs for a parameter whose backward returned ``None`` (the
    direct route; measured on the GPU path: every direct parameter reported twice,
    so buckets completed, and their all-reduce / optimizer update started, before
    their last gradient landed — ``tools/diag_grad_ready.py``).  That firing is
    skipped: it consumes the flag the direct notification left.  Returns the
    post-hook handle."""
    def acc(q):
        if getattr(q, "_kfa_direct", False):
            q._kfa_direct = False
            return
        hook(q)
    set_ready_callback(p, hook)
    return p.register_post_accumulate_grad_hook(acc)


def _round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


class FlatGroup:
    def __init__(self, params: Sequence[torch.nn.Parameter], *, pad_to: int = ALIGN, master: Optional[bool] = None,
                 name: str = ""):
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("FlatGroup: no trainable parameters")
        dtypes = {p.dtype for p in params}
        devices = {p.device for p in params}
        if len(dtypes) != 1 or len(devices) != 1:
            raise ValueError(f"FlatGroup needs one dtype/device, got {dtypes} / {devices}")
        self.name = name
        self.params: List[torch.nn.Parameter] = list(params)
        self.dtype = params[0].dtype
        self.device = params[0].device
        self.offsets: List[int] = []
        off = 0
        for p in self.params:
            if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError("FlatGroup: parameters must be dense (contiguous or channels_last)")
            self.offsets.append(off)
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = _round_up(max(off, 1), max(pad_to, ALIGN))
        self.data = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        for p, o in zip(self.params, self.offsets):
            view = torch.as_strided(self.data, p.shape, p.stride(), o)
            view.copy_(p.data)
            p.data = view
            p.grad = torch.as_strided(self.grad, p.shape, p.stride(), o)
            p._kfa_flat = True
        use_master = (self.dtype != torch.float32) if master is None else master
        self.master: Optional[torch.Tensor] = self.data.float() if use_master else None
        # fp32 gradient buffer the cross-rank sum runs in when the compute grads are
        # bf16 (set by ``parallel.ddp.GradSync``); the optimizer then reads it
        self.grad32: Optional[torch.Tensor] = None

    # the fp32 tensor the optimizer updates
    @property
    def fp32(self) -> torch.Tensor:
        return self.master if self.master is not None else self.data

    @property
    def opt_grad(self) -> torch.Tensor:
        """The gradient the optimizer consumes (the fp32 reduction buffer if one exists)."""
        return self.grad32 if self.grad32 is not None else self.grad

    def zero_grad(self) -> None:
        self.grad.zero_()
        # autograd may have replaced .grad (e.g. after a user set it to None): re-bind views
        for p, o in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + o * self.grad.element_size():
                p.grad = torch.as_strided(self.grad, p.shape, p.stride(), o)

    def param_range(self, i: int):
        return self.offsets[i], self.offsets[i] + self.params[i].numel()

    def __repr__(self) -> str:
        return f"FlatGroup({self.name!r}, {len(self.params)} tensors, {self.numel} x {self.dtype})"


def split_params(model: torch.nn.Module, compute_dtype=torch.bfloat16, pad_to: int = ALIGN) -> List[FlatGroup]:
    """Cast >=2-D weights to ``compute_dtype`` (bf16 with fp32 master) and keep
    1-D params (norm scales, biases) fp32; return one FlatGroup per dtype.

    Group names: ``"weights"`` (weight decay applies) and ``"norms_biases"``
    (no decay — the usual large-batch recipe)."""
    big, small = [], []
    # row-sharded tables: marked on the tensor and by their module's class (a
    # tensor attribute does not survive copy.deepcopy of the model)
    sparse = {id(p) for m in model.modules() if getattr(type(m), "kfa_sparse_module", False)
              for p in m.parameters(recurse=False)}
    for p in model.parameters():
        if not p.requires_grad or getattr(p, "_kfa_sparse", False) or id(p) in sparse:
            continue  # frozen, or a row-sharded table updated by its owner (parallel/embedding.py)
        if p.dim() >= 2 and compute_dtype is not None and p.dtype != compute_dtype:
            p.data = p.data.to(compute_dtype)
        (big if p.dim() >= 2 else small).append(p)
    for p in small:
        if p.dtype != torch.float32:
            p.data = p.data.float()
    groups = []
    if big:
        groups.append(FlatGroup(big, pad_to=pad_to, name="weights"))
    if small:
        groups.append(FlatGroup(small, pad_to=pad_to, name="norms_biases"))
    return groups


def group_bytes(groups: Sequence[FlatGroup]) -> Dict[str, int]:
    return {g.name: g.numel * g.grad.element_size() for g in groups}
