"""Fully connected layer: ``y = x · Wᵀ + b``.

On the GPU the layer runs through :class:`ops.transformer.DenseFn` — the
hand-written MFMA GEMM with the bias fused into its epilogue when
``KFA_GEMM=1`` routes dense layers to it (``ops/gemm.py``), else the library
GEMM plus ONE fused bias pass (``kfa_bias_act_fwd``); the backward's dbias is
the same kernel's column sums and dW the hand-written ``wgrad_kernel``
accumulating into the flat gradient.  Reference math:
``/root/reference/examples/workdir/mnist_replica.py:164-167`` (``xw_plus_b``),
``mnist_softmax.py:43`` (``matmul + b``).  Shapes the kernels do not take
(feature counts not multiples of 8, e.g. MNIST's 10 classes) and the CPU use
``F.linear``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def _kernel_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0
            and x.shape[-1] == w.shape[1])


class Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def forward(self, x):
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        if _kernel_ok(x, w):
            from . import transformer as T
            b = None if self.bias is None else (self.bias if self.bias.dtype == torch.float32 else self.bias.float())
            return T.dense(x.contiguous(), w, b)
        b = None if self.bias is None else self.bias.to(x.dtype)
        return F.linear(x, w, b)

    def extra_repr(self) -> str:
        return f"{self.in_features}, {self.out_features}, bias={self.bias is not None}"
