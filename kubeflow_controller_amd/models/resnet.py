"""ResNet-50 (v1.5: stride on the 3x3) in NHWC bf16 — the headline benchmark model.

BASELINE.json configs "ResNet-50 synthetic ImageNet ..." (SURVEY §2.6 K7/K8/K9/K1/K2).
Every BatchNorm is a fused ``BatchNorm2dAct`` (BN + optional residual add +
ReLU in one HIP kernel chain); the residual add and the block's final ReLU are
folded into ``bn3``.  Convolutions go through ``ops.conv.Conv2d`` (NHWC).
The last BN of each block is zero-initialised (standard large-batch recipe).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from ..ops.batchnorm import DS_SLOTS, BatchNorm2dAct, bn_act_dual, bn_relu_maxpool
from ..ops.conv import Conv2d, GradJoin
from ..ops.linear import Linear
from ..ops.pool import MaxPool2d, global_avg_pool


DUAL_BN = os.environ.get("KFA_BN_DUAL", "1") != "0"
# bn2's output (read only by the 1x1 conv3) is left lazy: conv3 folds the BN-apply + ReLU
# into its operand load where the per-shape tuner measured that faster (ops.conv._use_bnpro)
LAZY_BN2 = os.environ.get("KFA_LAZY_BN2", "1") != "0"
FUSED_STEM_POOL = os.environ.get("KFA_STEM_POOL_FUSED", "1") != "0"


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, mid: int, stride: int):
        super().__init__()
        cout = mid * self.expansion
        self.conv1 = Conv2d(cin, mid, 1)
        self.bn1 = BatchNorm2dAct(mid, relu=True)
        self.conv2 = Conv2d(mid, mid, 3, stride=stride, padding=1)
        self.bn2 = BatchNorm2dAct(mid, relu=True)
        self.conv3 = Conv2d(mid, cout, 1)
        self.bn3 = BatchNorm2dAct(cout, relu=True, zero_init=True)  # + residual, fused
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.ModuleDict({"conv": Conv2d(cin, cout, 1, stride=stride),
                                             "bn": BatchNorm2dAct(cout, relu=False)})

    def forward(self, x):
        # x feeds two branches; its gradient sum is fused into a dgrad epilogue
        # (ops.conv.GradJoin) instead of a separate add kernel.  In training every
        # conv accumulates its BatchNorm's statistics in its epilogue (st=True):
        # the BN then only finalizes + applies (no stats pass over the output).
        # bn1 / bn2 outputs feed exactly one conv (conv2 / conv3): their backward
        # statistics are accumulated in that conv's dgrad epilogue (bwd_link).
        # bn3's output (the block output) feeds the next block's conv1 (or
        # downsample conv) AND its residual: that conv's dgrad epilogue adds the
        # residual gradient (GradJoin), so it sees the FULL gradient and takes
        # bn3's backward statistics too.  In identity blocks bn3's backward does
        # not even write the residual gradient: it hands conv1's dgrad epilogue
        # its raw output gradient + ReLU bits (GradJoin.deposit_masked).  (The last block feeds the pooling head:
        # no conv takes the link, and its BN runs its own statistics pass.)
        join = GradJoin()
        st = self.training
        if self.downsample is None:
            y = self.bn1(self.conv1(x, join=join, bn_stats=st), bwd_link=st)
            y = self.bn2(self.conv2(y, bn_stats=st), bwd_link=st, lazy=st and LAZY_BN2)
            return self.bn3(self.conv3(y, bn_stats=st), residual=join.branch(x), bwd_link=st, res_join=join)
        # downsample block: relu(bn3(.) + bn_ds(.)) in ONE apply pass each way
        # (ops.batchnorm.bn_act_dual): the downsample conv's statistics wait in
        # their own slot workspace while conv1..conv3 fill the shared one.
        dual = DUAL_BN and st and x.is_cuda
        r = self.downsample["conv"](x, join=join, bn_stats=(DS_SLOTS if dual else st))
        idn = None if dual else self.downsample["bn"](r)
        y = self.bn1(self.conv1(join.branch(x), bn_stats=st), bwd_link=st)
        y = self.bn2(self.conv2(y, bn_stats=st), bwd_link=st, lazy=st and LAZY_BN2)
        if dual:
            return bn_act_dual(self.bn3, self.conv3(y, bn_stats=st), self.downsample["bn"], r, bwd_link=st)
        return self.bn3(self.conv3(y, bn_stats=st), residual=idn, bwd_link=st)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.conv1 = Conv2d(3, width, 7, stride=2, padding=3)
        self.bn1 = BatchNorm2dAct(width, relu=True)
        self.maxpool = MaxPool2d(3, 2, 1)
        blocks = []
        cin = width
        for i, n in enumerate(layers):
            mid = width * (2 ** i)
            for j in range(n):
                blocks.append(Bottleneck(cin, mid, (1 if i == 0 else 2) if j == 0 else 1))
                cin = mid * Bottleneck.expansion
        self.layers = nn.Sequential(*blocks)
        self.fc = Linear(cin, num_classes)
        self.reset_parameters()

    def reset_parameters(self):
        for m in self.modules():
            if isinstance(m, Conv2d):
                fan_out = m.out_channels * m.kernel_size * m.kernel_size
                nn.init.normal_(m.weight, 0.0, math.sqrt(2.0 / fan_out))
        nn.init.normal_(self.fc.weight, 0.0, 0.01)
        nn.init.zeros_(self.fc.bias)

    def forward(self, x):
        x = self.conv1(x, bn_stats=self.training)
        # stem BN + ReLU + 3x3/s2 max pool: one pass over the conv output in training
        x = bn_relu_maxpool(self.bn1, x) if FUSED_STEM_POOL else self.maxpool(self.bn1(x))
        x = self.layers(x)
        return self.fc(global_avg_pool(x))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)


def resnet_tiny(num_classes: int = 10) -> ResNet:
    """Same code path, toy width — for CPU plumbing tests and smoke()."""
    return ResNet((1, 1, 1, 1), num_classes, width=8)
