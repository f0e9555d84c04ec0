"""Softmax cross-entropy (fwd+bwd fused) and argmax/accuracy — ``csrc/kernels/loss.hip``.

SURVEY §2.6 K2/K3: replaces ``softmax`` + clip + log + reduce_sum of
``mnist_replica.py:167-168`` and ``softmax_cross_entropy_with_logits`` of
``mnist_softmax.py:57-58``; at ResNet/BERT scale the gradient is produced in
the same kernel as the loss so backward launches nothing.
"""
from __future__ import annotations

import math

import torch

from . import _lib

_lib.register("kfa_softmax_xent", [_lib.P, _lib.I, _lib.P, _lib.P, _lib.P, _lib.P, _lib.L, _lib.I, _lib.F, _lib.F,
                                    _lib.P])
_lib.register("kfa_argmax", [_lib.P, _lib.I, _lib.P, _lib.L, _lib.I, _lib.P])
_lib.register("kfa_cls_head_blocks", [_lib.I])
_lib.register("kfa_cls_head_fwd", [_lib.P] * 7 + [_lib.I] * 3 + [_lib.P])
_lib.register("kfa_cls_head_bwd", [_lib.P] * 8 + [_lib.I] * 3 + [_lib.P])


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing):
        z = logits.contiguous()
        rows, V = z.numel() // z.shape[-1], z.shape[-1]
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        if lab.numel() != rows:
            raise ValueError(f"cross_entropy: {lab.numel()} labels for {rows} rows")
        row_loss = torch.empty(rows, dtype=torch.float32, device=z.device)
        dz = torch.empty_like(z) if logits.requires_grad else None
        valid = max(int(rows), 1)
        _lib.call("kfa_softmax_xent", _lib.ptr(z), int(z.dtype == torch.bfloat16), _lib.ptr(lab), None, _lib.ptr(row_loss),
                  _lib.ptr(dz), rows, V, 1.0 / valid, float(smoothing), _lib.stream())
        ctx.save_for_backward(dz)
        return row_loss.sum() / valid

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return dz * g.to(dz.dtype), None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, label_smoothing: float = 0.0) -> torch.Tensor:
    """Mean softmax cross-entropy over rows; fp32 scalar loss."""
    if not logits.is_cuda:
        return torch.nn.functional.cross_entropy(logits.float(), labels, label_smoothing=label_smoothing)
    if logits.dtype not in (torch.bfloat16, torch.float32):
        logits = logits.float()
    return _XentFn.apply(logits, labels, label_smoothing)


class _ClsHeadXentFn(torch.autograd.Function):
    """``mean CE(x @ W.T + b, labels)`` for a small classifier (C <= 8 classes,
    e.g. BERT's NSP head) in one HIP pass each way (``csrc/kernels/loss.hip``
    ``cls_head_*``): no N = C GEMM on the library, no logits tensor."""

    @staticmethod
    def forward(ctx, x, w, b, labels):
        B, H = x.shape
        C = w.shape[0]
        w32 = w.detach().float().contiguous()
        b32 = b.detach().float().reshape(-1).contiguous()
        y = labels.reshape(-1).to(torch.int64).contiguous()
        prob = torch.empty(B, C, dtype=torch.float32, device=x.device)
        part = torch.empty(_lib.lib().kfa_cls_head_blocks(B), dtype=torch.float32, device=x.device)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        _lib.call("kfa_cls_head_fwd", _lib.ptr(x), _lib.ptr(w32), _lib.ptr(b32), _lib.ptr(y), _lib.ptr(prob),
                  _lib.ptr(part), _lib.ptr(loss), B, H, C, _lib.stream())
        ctx.save_for_backward(x, w32, y, prob)
        ctx.meta = (w.shape, w.dtype, b.shape, b.dtype)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, w32, y, prob = ctx.saved_tensors
        wshape, wdt, bshape, bdt = ctx.meta
        B, H = x.shape
        C = w32.shape[0]
        dl = g.detach().float().reshape(1).contiguous()
        dx = torch.empty_like(x)
        nb = _lib.lib().kfa_cls_head_blocks(B)
        part = _lib.workspace(4 * nb * (C * H + C), x.device, "cls_head_part")
        grads = torch.empty(C * H + C, dtype=torch.float32, device=x.device)
        _lib.call("kfa_cls_head_bwd", _lib.ptr(x), _lib.ptr(w32), _lib.ptr(y), _lib.ptr(prob), _lib.ptr(dl), _lib.ptr(dx),
                  _lib.ptr(part), _lib.ptr(grads), B, H, C, _lib.stream())
        return dx, grads[:C * H].view(wshape).to(wdt), grads[C * H:].view(bshape).to(bdt), None


def classifier_xent(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy of the classifier ``x @ w.T + b`` (fp32 scalar):
    the fused HIP head for bf16 ``x`` with C <= 8 classes, else the PyTorch ops."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.is_contiguous() and x.data_ptr() % 16 == 0
            and 0 < w.shape[0] <= 8 and x.shape[1] % 8 == 0 and x.shape[1] <= 1024 and w.shape[1] == x.shape[1]
            and w.shape[0] * x.shape[1] <= 4096):  # the backward's per-block LDS image: 8 x (C·H + C) floats
        return _ClsHeadXentFn.apply(x, w, b, labels)
    logits = x.float() @ w.float().t() + b.float()
    return torch.nn.functional.cross_entropy(logits, labels.reshape(-1))


class _ClippedSumXentFn(torch.autograd.Function):
    """Summed cross-entropy of clipped probabilities, one fused kernel pass: the
    kernel's per-row loss and ``softmax - onehot`` gradient at scale 1, then the
    rows whose label probability fell under the clip (loss > -log eps) lose their
    gradient and are capped — ``tf.clip_by_value`` passes no gradient there."""

    @staticmethod
    def forward(ctx, logits, labels, eps):
        z = logits.contiguous()
        rows, V = z.numel() // z.shape[-1], z.shape[-1]
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        if lab.numel() != rows:
            raise ValueError(f"clipped_sum_cross_entropy: {lab.numel()} labels for {rows} rows")
        row_loss = torch.empty(rows, dtype=torch.float32, device=z.device)
        dz = torch.empty_like(z) if logits.requires_grad else None
        _lib.call("kfa_softmax_xent", _lib.ptr(z), int(z.dtype == torch.bfloat16), _lib.ptr(lab), None,
                  _lib.ptr(row_loss), _lib.ptr(dz), rows, V, 1.0, 0.0, _lib.stream())
        cap = -math.log(eps)
        clipped = row_loss > cap
        if dz is not None:
            dz.view(rows, V).masked_fill_(clipped.view(rows, 1), 0)
        ctx.save_for_backward(dz)
        return row_loss.clamp(max=cap).sum()

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return dz * g.to(dz.dtype), None, None


def clipped_sum_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, eps: float = 1e-10) -> torch.Tensor:
    """``-Σ y · log(clip(softmax(z), eps, 1))`` summed over the batch: the loss the
    reference's distributed MNIST minimises (``mnist_replica.py:167-168``), where
    :func:`cross_entropy` is the batch mean of ``mnist_softmax.py:57-58``."""
    if not logits.is_cuda:
        p = torch.softmax(logits.float(), -1)
        return -torch.log(p.gather(-1, labels.reshape(-1, 1).long()).clamp(eps, 1.0)).sum()
    if logits.dtype not in (torch.bfloat16, torch.float32):
        logits = logits.float()
    return _ClippedSumXentFn.apply(logits, labels, float(eps))


def argmax(logits: torch.Tensor) -> torch.Tensor:
    if not logits.is_cuda:
        return logits.argmax(-1)
    z = logits.contiguous()
    if z.dtype not in (torch.bfloat16, torch.float32):
        z = z.float()
    rows, V = z.numel() // z.shape[-1], z.shape[-1]
    out = torch.empty(rows, dtype=torch.int64, device=z.device)
    _lib.call("kfa_argmax", _lib.ptr(z), int(z.dtype == torch.bfloat16), _lib.ptr(out), rows, V, _lib.stream())
    return out.view(z.shape[:-1])


def accuracy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """``mean(argmax(z) == y)`` (``mnist_softmax.py:70-71``)."""
    return (argmax(logits) == labels.reshape(argmax(logits).shape)).float().mean()
