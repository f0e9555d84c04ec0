"""MNIST models of the reference workloads + a synthetic MNIST.

* ``MnistSoftmax``: 784 -> 10 linear + softmax cross-entropy, GD lr 0.5, batch 100
  (``examples/workdir/mnist_softmax.py:35-73``).
* ``MnistMLP``: 784 -> hidden(100) ReLU -> 10, Adam lr 0.01, batch 100
  (``examples/workdir/mnist_replica.py:142-184``).

There is no network here, so ``SyntheticMNIST`` generates a learnable stand-in:
10 fixed random 28x28 class prototypes, each sample = its class prototype +
noise, pixel range [0, 1].  Same shapes and dtypes as ``input_data.read_data_sets``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.linear import Linear


class MnistSoftmax(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.fc = Linear(784, num_classes)
        nn.init.zeros_(self.fc.weight)  # tf.zeros init (mnist_softmax.py:43-44)

    def forward(self, x):
        return self.fc(x.reshape(x.shape[0], -1))


class MnistMLP(nn.Module):
    def __init__(self, hidden_units: int = 100, num_classes: int = 10):
        super().__init__()
        self.hid = Linear(784, hidden_units)
        self.sm = Linear(hidden_units, num_classes)
        # truncated_normal(stddev=1/sqrt(fan_in)) (mnist_replica.py:145-158)
        for lin, fan in ((self.hid, 784), (self.sm, hidden_units)):
            nn.init.trunc_normal_(lin.weight, std=1.0 / fan ** 0.5, a=-2.0 / fan ** 0.5, b=2.0 / fan ** 0.5)
            nn.init.zeros_(lin.bias)

    def forward(self, x):
        return self.sm(torch.relu(self.hid(x.reshape(x.shape[0], -1))))


class SyntheticMNIST:
    def __init__(self, n_train: int = 55000, n_val: int = 5000, n_test: int = 10000, seed: int = 1234,
                 noise: float = 3.0):
        g = torch.Generator().manual_seed(seed)
        self.protos = (torch.rand(10, 784, generator=g) > 0.75).float()
        self.noise = noise
        self._g = torch.Generator().manual_seed(seed + 1)
        self.train = self._make(n_train, g)
        self.validation = self._make(n_val, g)
        self.test = self._make(n_test, g)
        self._pos = 0
        self._perm = None  # epoch order after the first pass (indices; the split itself is never re-laid out)

    def _make(self, n, g):
        y = torch.randint(0, 10, (n,), generator=g)
        x = (self.protos[y] + self.noise * torch.randn(n, 784, generator=g)).clamp_(0, 1)
        return x, y

    def to(self, device) -> "SyntheticMNIST":
        """Keep the splits resident on ``device`` (no host copy per step)."""
        self.train = tuple(t.to(device) for t in self.train)
        self.validation = tuple(t.to(device) for t in self.validation)
        self.test = tuple(t.to(device) for t in self.test)
        return self

    def next_batch(self, batch_size: int):
        """Next ``batch_size`` examples; each epoch after the first visits the split in
        a fresh random order (``input_data``'s shuffle) by gathering the batch's rows."""
        x, y = self.train
        if self._pos + batch_size > x.shape[0]:
            self._perm = torch.randperm(x.shape[0], generator=self._g).to(x.device)
            self._pos = 0
        s = slice(self._pos, self._pos + batch_size)
        self._pos += batch_size
        if self._perm is None:
            return x[s], y[s]
        idx = self._perm[s]
        return x.index_select(0, idx), y.index_select(0, idx)
