"""Pooling: NHWC bf16 max pool (HIP, ``csrc/kernels/pool.hip``)
and global average pool (head)."""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_lib.register("kfa_maxpool_fwd", [_lib.P, _lib.P, _lib.P] + [_lib.I] * 9 + [_lib.P])
_lib.register("kfa_maxpool_bwd", [_lib.P, _lib.P, _lib.P] + [_lib.I] * 9 + [_lib.P])
_lib.register("kfa_gap_fwd", [_lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.P])
_lib.register("kfa_gap_bwd", [_lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.P])


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        Ho = (H + 2 * p - k) // s + 1
        Wo = (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((N, C, Ho, Wo), dtype=torch.uint8, device=x.device, memory_format=torch.channels_last)
        _lib.call("kfa_maxpool_fwd", _lib.ptr(x), _lib.ptr(y), _lib.ptr(idx), N, H, W, C, Ho, Wo, k, s, p,
                  _lib.stream())
        ctx.save_for_backward(idx)
        ctx.meta = (N, C, H, W, Ho, Wo, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.call("kfa_maxpool_bwd", _lib.ptr(dy), _lib.ptr(idx), _lib.ptr(dx), N, H, W, C, Ho, Wo, k, s, p,
                  _lib.stream())
        return dx, None, None, None


def max_pool2d(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1) -> torch.Tensor:
    if x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0:
        return _MaxPoolFn.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p)


class MaxPool2d(nn.Module):
    def __init__(self, kernel_size: int = 3, stride: int = 2, padding: int = 1):
        super().__init__()
        self.k, self.s, self.p = kernel_size, stride, padding

    def forward(self, x):
        return max_pool2d(x, self.k, self.s, self.p)


HIP_GAP = os.environ.get("KFA_HIP_GAP", "1") != "0"


class _GapFn(torch.autograd.Function):
    """Global average pool over NHWC bf16 (``kfa_gap_fwd`` / ``kfa_gap_bwd``): the
    backward writes dy / HW straight into an NHWC gradient in one pass."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous(memory_format=torch.channels_last)
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=x.dtype, device=x.device)
        _lib.call("kfa_gap_fwd", _lib.ptr(x), _lib.ptr(y), N, H * W, C, _lib.stream())
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.call("kfa_gap_bwd", _lib.ptr(dy), _lib.ptr(dx), N, H * W, C, _lib.stream())
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (NHWC memory) -> [N, C], fp32 accumulation (HIP on bf16 CUDA input)."""
    if HIP_GAP and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0:
        return _GapFn.apply(x)
    return x.mean((2, 3), dtype=torch.float32).to(x.dtype)
