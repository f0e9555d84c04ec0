"""Fused BatchNorm(+residual)(+ReLU) for NHWC bf16 — HIP kernel ``csrc/kernels/batchnorm.hip``.

SURVEY §2.6 K8.  On a stock PyTorch-ROCm ResNet-50 step the channels-last BN
kernels plus the separate ReLU/add elementwise kernels cost 57 of 74 ms
(``profiles/r0_stock_torch_resnet50_bs256.md``); this op replaces all of them
with 3 streaming passes forward and 3 backward.

Layout contract: ``x`` is a 4-D bf16 tensor in channels_last memory format (or
any tensor whose memory is ``[M, C]`` row-major with C innermost); params are
fp32.  Without a residual the backward's ReLU mask is recomputed from the
input and the layer's saved [scale | shift] (2C floats); with one, the forward
also writes the mask as bits (1/16 of the output's bytes).  Either way the backward
never reads the output (env ``KFA_BN_MASK_FROM_X=0`` reads it instead).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import _lib
from ..parallel.flat import direct_grad_view, notify_grad_ready


MASK_FROM_X = os.environ.get("KFA_BN_MASK_FROM_X", "1") != "0"


def _as_rows(t: torch.Tensor) -> torch.Tensor:
    """Check that ``t``'s memory is [M, C] with C innermost (NHWC / 2-D)."""
    if t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            t = t.contiguous(memory_format=torch.channels_last)
    elif not t.is_contiguous():
        t = t.contiguous()
    return t


def _mc(t: torch.Tensor):
    C = t.shape[1] if t.dim() == 4 else t.shape[-1]
    return t.numel() // C, C


_lib.register("kfa_bn_fwd_train_prestats", [_lib.P] * 11 + [_lib.L, _lib.I, _lib.F, _lib.F, _lib.I, _lib.P, _lib.P])
_lib.register("kfa_bn_bwd_prestats", [_lib.P] * 12 + [_lib.L, _lib.I, _lib.I, _lib.I, _lib.P, _lib.P, _lib.P])
_lib.register("kfa_bn_finalize", [_lib.P, _lib.P, _lib.L, _lib.I] + [_lib.P] * 7 + [_lib.F, _lib.F, _lib.I, _lib.P])
_lib.register("kfa_bn_fwd_train_dual", [_lib.P] * 11 + [_lib.L, _lib.I, _lib.F, _lib.F, _lib.I, _lib.P, _lib.P,
                                                        _lib.I, _lib.P])
_lib.register("kfa_bn_bwd_rstats", [_lib.P] * 11 + [_lib.L, _lib.I, _lib.I, _lib.I] + [_lib.P] * 5 + [_lib.I, _lib.P])
_lib.register("kfa_bn_apply_ss", [_lib.P, _lib.P, _lib.P, _lib.L, _lib.I, _lib.I, _lib.P])


class LazyBN:
    """A training BatchNorm + ReLU whose apply pass is deferred to its consumer: the
    output tensor is allocated but NOT written; ``x`` (the BN input) and ``ss`` (its
    [scale | shift]) let the one convolution that reads it fold relu(x·scale + shift)
    into its A-operand load (``ops.conv.conv_fwd_bnpro``, which also fills the output
    for the weight gradient), or :func:`materialize` runs the apply pass first.  Only a
    model that guarantees that conv is the sole reader may ask for it (``lazy=True``)."""

    __slots__ = ("x", "ss", "pending")

    def __init__(self):
        self.x = self.ss = None
        self.pending = False


def materialize(t: torch.Tensor) -> torch.Tensor:
    """Write a lazy BatchNorm output (no-op for any other tensor)."""
    lz = getattr(t, "_kfa_lazy", None)
    if lz is not None and lz.pending:
        M, C = _mc(lz.x)
        _lib.call("kfa_bn_apply_ss", _lib.ptr(lz.x), _lib.ptr(t), _lib.ptr(lz.ss), M, C, 1, _lib.stream())
        lz.pending = False
    return t


class BnBwdLink:
    """Hand-off from a BatchNorm to the ONE convolution consuming its output: the
    conv's dgrad epilogue accumulates this BN's backward statistics (sum dz,
    sum dz*(x-mean)) into the BN slots and sets ``prestats``; the BN backward
    then skips its statistics pass.  Only valid when that conv is the sole
    consumer of the BN output's gradient: the model decides (ResNet bn1/bn2, and
    bn3 whose other consumer, the residual, hands its gradient to that conv's
    epilogue through a ``GradJoin``).  ``convs`` counts the convolutions that
    took the output as input; with more than one, none of them uses the link."""

    __slots__ = ("x", "y", "ss", "mb", "mean", "relu", "prestats", "convs")

    def __init__(self):
        self.x = self.y = self.ss = self.mb = self.mean = None
        self.relu = False
        self.prestats = False
        self.convs = 0


def bn_slot_workspace(C: int, device, tag: str = "bn_slots") -> torch.Tensor:
    """The zero-initialised, self-cleaning statistics slots shared by every BN
    (and by convolutions that accumulate a BN's statistics in their epilogue).
    ``DS_SLOTS``: a second set for the downsample BN of :func:`bn_act_dual`,
    whose statistics wait there while the block's other BNs use the first."""
    return _lib.workspace(_lib.lib().kfa_bn_slot_floats(C) * 4, device, tag)


DS_SLOTS = "bn_slots_ds"


def _workspaces(C: int, device):
    L = _lib.lib()
    slots = _lib.workspace(L.kfa_bn_slot_floats(C) * 4, device, "bn_slots")  # zero-init, self-cleaning
    coef = _lib.workspace(L.kfa_bn_coef_floats(C) * 4, device, "bn_coef")
    return slots, coef


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, training, momentum, eps, relu,
                prestats=False, link=None, res_join=None, lazy=None):
        x = _as_rows(x)
        M, C = _mc(x)
        if x.dtype != torch.bfloat16:
            raise TypeError("bn_act: bf16 activations required")
        res = _as_rows(residual) if residual is not None else None
        if res is not None and (res.shape != x.shape or res.dtype != x.dtype):
            raise ValueError(f"bn_act: residual {tuple(res.shape)} does not match input {tuple(x.shape)}")
        y = torch.empty_like(x)
        slots, coef = _workspaces(C, x.device)
        s = _lib.stream()
        ss = mb = None
        if training:
            mean = torch.empty(C, dtype=torch.float32, device=x.device)
            invstd = torch.empty_like(mean)
            if relu and res is None and MASK_FROM_X:
                # keep this layer's [scale | shift]: the backward recomputes the ReLU
                # mask from x instead of reading y (2 of its 8 bytes per element)
                ss = torch.empty(2 * C, dtype=torch.float32, device=x.device)
            elif relu and MASK_FROM_X:
                # with a residual the mask needs the output: keep it as bits (1/16 of y)
                mb = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device)
            if lazy is not None and ss is not None:  # finalize only: the consumer conv applies it
                _lib.call("kfa_bn_finalize", _lib.ptr(x), _lib.ptr(slots), M, C, _lib.ptr(weight), _lib.ptr(bias),
                          _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(mean), _lib.ptr(invstd),
                          _lib.ptr(ss), eps, momentum, int(prestats), s)
                lazy.x, lazy.ss, lazy.pending = x, ss, True
            else:
                _lib.call("kfa_bn_fwd_train_prestats" if prestats else "kfa_bn_fwd_train", _lib.ptr(x),
                          _lib.ptr(res), _lib.ptr(y), _lib.ptr(weight), _lib.ptr(bias),
                          _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(mean), _lib.ptr(invstd),
                          _lib.ptr(slots), _lib.ptr(coef if ss is None else ss), M, C, eps, momentum, int(relu),
                          _lib.ptr(mb), s)
        else:
            _lib.call("kfa_bn_fwd_eval", _lib.ptr(x), _lib.ptr(res), _lib.ptr(y), _lib.ptr(weight), _lib.ptr(bias),
                      _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(coef), M, C, eps, int(relu), s)
            var = running_var
            mean = running_mean.clone()
            invstd = torch.rsqrt(var + eps)
        ymask = y if (relu and ss is None and mb is None) else None
        ctx.save_for_backward(x, ymask, ss, mb, weight, mean, invstd)
        ctx.link = link if training else None
        if ctx.link is not None:
            link.x, link.y, link.ss, link.mb, link.mean = x, ymask, ss, mb, mean
            link.relu, link.prestats = bool(relu), False
        ctx.relu = relu
        ctx.has_res = residual is not None
        # residual = a GradJoin branch whose consumer conv can apply the ReLU bits
        # itself: the backward then skips writing dres (2 of its ~8 bytes per element)
        ctx.res_join = res_join if (training and mb is not None and residual is not None) else None
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, ss, mb, weight, mean, invstd = ctx.saved_tensors
        dy = _as_rows(dy)
        M, C = _mc(x)
        dx = torch.empty_like(x)
        deposited = ctx.res_join is not None and ctx.res_join.deposit_masked(dy, mb)
        dres = torch.empty_like(x) if (ctx.has_res and not deposited) else None
        need_w = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        direct = False
        dgamma = dbeta = None
        if need_w:
            gv, bv = ctx.params
            wv, bvv = direct_grad_view(gv), direct_grad_view(bv)
            if wv is not None and bvv is not None and wv.dtype == torch.float32 and bvv.dtype == torch.float32:
                dgamma, dbeta, direct = wv, bvv, True  # += straight into the flat grad bucket
            else:
                dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
                dbeta = torch.empty(C, dtype=torch.float32, device=x.device)
        slots, coef = _workspaces(C, x.device)
        lk = ctx.link
        pre = lk is not None and lk.prestats
        if lk is not None:
            lk.prestats = False
            lk.x = lk.y = lk.ss = lk.mb = lk.mean = None
        _lib.call("kfa_bn_bwd_prestats" if pre else "kfa_bn_bwd", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(y), _lib.ptr(weight), _lib.ptr(mean),
                  _lib.ptr(invstd), _lib.ptr(dx), _lib.ptr(dres), _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(slots),
                  _lib.ptr(coef),
                  M, C, int(ctx.relu), int(direct), _lib.ptr(ss), _lib.ptr(mb), _lib.stream())
        if direct:
            notify_grad_ready(ctx.params[0])
            notify_grad_ready(ctx.params[1])
            return dx, None, None, None, None, dres, None, None, None, None, None, None, None, None
        if dgamma is not None and weight is not None and weight.dtype != torch.float32:
            dgamma, dbeta = dgamma.to(weight.dtype), dbeta.to(weight.dtype)
        return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None


def bn_act(x, weight, bias, running_mean, running_var, residual=None, training=True, momentum=0.1, eps=1e-5,
           relu=True, prestats=False, bwd_link=False, res_join=None, lazy=False):
    """``prestats``: the statistics of ``x`` already sit in the BN slot workspace
    (accumulated by the producing convolution's epilogue).  ``bwd_link``: the
    output feeds exactly one igemm convolution, whose dgrad epilogue may compute
    this BN's backward statistics (``BnBwdLink``).  ``res_join``: the ``ops.conv.GradJoin``
    whose branch ``residual`` is; the backward then deposits the raw output
    gradient and the ReLU bits there instead of writing the residual gradient."""
    if prestats and not training:  # never leave the self-cleaning slots dirty
        bn_slot_workspace(x.shape[1], x.device).zero_()
        prestats = False
    link = BnBwdLink() if (bwd_link and training) else None
    lz = LazyBN() if (lazy and training and relu and residual is None and MASK_FROM_X and x.is_cuda) else None
    y = _BNActFn.apply(x, weight, bias, running_mean, running_var, residual, training, momentum, eps, relu,
                       prestats, link, res_join, lz)
    if link is not None:
        y._kfa_bn_link = link
    if lz is not None and lz.pending:
        y._kfa_lazy = lz
    return y


def _param_grads(weight, bias, C, device):
    """(dgamma, dbeta, direct): views into the flat fp32 gradient bucket when the
    params live there (the kernel then accumulates), else fresh fp32 vectors."""
    wv, bv = direct_grad_view(weight), direct_grad_view(bias)
    if wv is not None and bv is not None and wv.dtype == torch.float32 and bv.dtype == torch.float32:
        return wv, bv, True
    return (torch.empty(C, dtype=torch.float32, device=device), torch.empty(C, dtype=torch.float32, device=device),
            False)


class _BNDualFn(torch.autograd.Function):
    """``relu(bn(x) + bn_r(r))`` in training — a ResNet downsample block's tail
    (bn3 of the main branch plus the downsample BN of the shortcut).

    Forward: bn_r's statistics (accumulated by the downsample conv's epilogue
    into the ``DS_SLOTS`` workspace) are finalized into its [scale | shift];
    bn's apply pass normalises r itself (``bn_apply`` RAFF), so bn_r's output is
    never written or re-read.  Backward: bn's apply pass accumulates bn_r's
    statistics (``bn_bwd_apply_rstats``) instead of writing the shortcut
    gradient; bn_r's backward then re-derives that gradient from dy and the
    block output's ReLU bits.  Saves, per block, bn_r's forward apply pass and
    its backward statistics pass over a written residual gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, r, rweight, rbias, rrunning_mean, rrunning_var,
                momentum, eps, relu, prestats, rprestats, link):
        x, r = _as_rows(x), _as_rows(r)
        M, C = _mc(x)
        if x.dtype != torch.bfloat16 or r.dtype != torch.bfloat16 or r.shape != x.shape:
            raise ValueError(f"bn_act_dual: bf16 x {tuple(x.shape)} and r {tuple(r.shape)} of one shape required")
        dev = x.device
        s = _lib.stream()
        slots, coef = _workspaces(C, dev)
        rslots = bn_slot_workspace(C, dev, DS_SLOTS)
        f32 = dict(dtype=torch.float32, device=dev)
        rmean, rinv, rss = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(2 * C, **f32)
        _lib.call("kfa_bn_finalize", _lib.ptr(r), _lib.ptr(rslots), M, C, _lib.ptr(rweight), _lib.ptr(rbias),
                  _lib.ptr(rrunning_mean), _lib.ptr(rrunning_var), _lib.ptr(rmean), _lib.ptr(rinv), _lib.ptr(rss),
                  eps, momentum, int(rprestats), s)
        y = torch.empty_like(x)
        mean, invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        mb = torch.empty(M * C // 8, dtype=torch.uint8, device=dev) if relu else None
        _lib.call("kfa_bn_fwd_train_dual", _lib.ptr(x), _lib.ptr(r), _lib.ptr(y), _lib.ptr(weight), _lib.ptr(bias),
                  _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(slots),
                  _lib.ptr(coef), M, C, eps, momentum, int(relu), _lib.ptr(mb), _lib.ptr(rss), int(prestats), s)
        ctx.save_for_backward(x, r, mb, weight, rweight, mean, invstd, rmean, rinv)
        ctx.link = link
        if link is not None:
            link.x, link.y, link.ss, link.mb, link.mean = x, None, None, mb, mean
            link.relu, link.prestats = bool(relu), False
        ctx.relu = relu
        ctx.params = (weight, bias, rweight, rbias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, r, mb, weight, rweight, mean, invstd, rmean, rinv = ctx.saved_tensors
        dy = _as_rows(dy)
        M, C = _mc(x)
        dev = x.device
        s = _lib.stream()
        w, b, rw, rb = ctx.params
        dg, db, direct = _param_grads(w, b, C, dev)
        rdg, rdb, rdirect = _param_grads(rw, rb, C, dev)
        slots, coef = _workspaces(C, dev)
        rslots = bn_slot_workspace(C, dev, DS_SLOTS)
        lk = ctx.link
        pre = lk is not None and lk.prestats
        if lk is not None:
            lk.prestats = False
            lk.x = lk.y = lk.ss = lk.mb = lk.mean = None
        dx, dr = torch.empty_like(x), torch.empty_like(r)
        _lib.call("kfa_bn_bwd_rstats", _lib.ptr(dy), _lib.ptr(x), None, _lib.ptr(weight), _lib.ptr(mean),
                  _lib.ptr(invstd), _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(slots), _lib.ptr(coef), M, C,
                  int(ctx.relu), int(direct), None, _lib.ptr(mb), _lib.ptr(r), _lib.ptr(rmean), _lib.ptr(rslots),
                  int(pre), s)
        # bn_r: statistics now in rslots; dz = dy * (block output > 0) from the bits
        _lib.call("kfa_bn_bwd_prestats", _lib.ptr(dy), _lib.ptr(r), None, _lib.ptr(rweight), _lib.ptr(rmean),
                  _lib.ptr(rinv), _lib.ptr(dr), None, _lib.ptr(rdg), _lib.ptr(rdb), _lib.ptr(rslots), _lib.ptr(coef),
                  M, C, int(ctx.relu), int(rdirect), None, _lib.ptr(mb), s)
        out = []
        for p, g, d in ((w, dg, direct), (b, db, direct), (rw, rdg, rdirect), (rb, rdb, rdirect)):
            if d:
                notify_grad_ready(p)
                out.append(None)
            else:
                out.append(g if p.dtype == torch.float32 else g.to(p.dtype))
        return (dx, out[0], out[1], None, None, dr, out[2], out[3], None, None, None, None, None, None, None, None)


def bn_act_dual(bn: "BatchNorm2dAct", x: torch.Tensor, bn_r: "BatchNorm2dAct", r: torch.Tensor,
                bwd_link: bool = False) -> torch.Tensor:
    """``act(bn(x) + bn_r(r))`` with one apply pass each way (training, CUDA);
    ``bn_r`` must not have a ReLU of its own.  ``r``'s statistics may sit in the
    ``DS_SLOTS`` workspace (its conv ran with ``bn_stats=DS_SLOTS``).  Other
    cases run the two BNs separately."""
    if not (x.is_cuda and bn.training and bn_r.training and not bn_r.relu and bn.eps == bn_r.eps
            and bn.momentum == bn_r.momentum):
        if getattr(r, "_kfa_prestats_tag", None) == DS_SLOTS:  # never leave the slots dirty
            bn_slot_workspace(r.shape[1], r.device, DS_SLOTS).zero_()
            r._kfa_prestats = False  # bn_r runs its own statistics pass
        return bn(x, residual=bn_r(r), bwd_link=bwd_link)
    link = BnBwdLink() if bwd_link else None
    rpre = getattr(r, "_kfa_prestats", False) and getattr(r, "_kfa_prestats_tag", None) == DS_SLOTS
    if getattr(r, "_kfa_prestats", False) and not rpre:
        raise ValueError("bn_act_dual: r's statistics must be accumulated into the DS_SLOTS workspace")
    y = _BNDualFn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, r, bn_r.weight, bn_r.bias,
                        bn_r.running_mean, bn_r.running_var, bn.momentum, bn.eps, bn.relu,
                        getattr(x, "_kfa_prestats", False), rpre, link)
    if link is not None:
        y._kfa_bn_link = link
    return y


_lib.register("kfa_maxpool_fwd_bn", [_lib.P, _lib.P, _lib.P] + [_lib.I] * 9 + [_lib.P, _lib.P])
_lib.register("kfa_maxpool_bwd", [_lib.P, _lib.P, _lib.P] + [_lib.I] * 9 + [_lib.P])
_lib.register("kfa_maxpool_bwd_bnstats", [_lib.P, _lib.P, _lib.P] + [_lib.I] * 7 + [_lib.P] * 5)
# KFA_POOL_BN_STATS=0: the stem BN's backward statistics in their own pass instead of
# accumulated by the pool-gradient kernel (64-channel stems)
POOL_BN_STATS = os.environ.get("KFA_POOL_BN_STATS", "1") != "0"


class _BNReluPoolFn(torch.autograd.Function):
    """``maxpool(relu(bn(x)))`` for the ResNet stem (training): BN finalize, then
    ONE pass that normalises each window element and pools it (``kfa_maxpool_fwd_bn``)
    — the 4x larger BN output is never written or re-read.  Backward: the pool's
    gradient scatter, then the BN backward with the ReLU mask recomputed from x
    and the saved [scale | shift] (exactly what the unfused pair runs)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, prestats, k, s, p):
        x = _as_rows(x)
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        slots, _ = _workspaces(C, dev)
        f32 = dict(dtype=torch.float32, device=dev)
        mean, invstd, ss = torch.empty(C, **f32), torch.empty(C, **f32), torch.empty(2 * C, **f32)
        st = _lib.stream()
        _lib.call("kfa_bn_finalize", _lib.ptr(x), _lib.ptr(slots), M, C, _lib.ptr(weight), _lib.ptr(bias),
                  _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(ss),
                  eps, momentum, int(prestats), st)
        cl = torch.channels_last
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=dev, memory_format=cl)
        idx = torch.empty((N, C, Ho, Wo), dtype=torch.uint8, device=dev, memory_format=cl)
        _lib.call("kfa_maxpool_fwd_bn", _lib.ptr(x), _lib.ptr(y), _lib.ptr(idx), N, H, W, C, Ho, Wo, k, s, p,
                  _lib.ptr(ss), st)
        ctx.save_for_backward(x, ss, idx, weight, mean, invstd)
        ctx.meta = (N, C, H, W, Ho, Wo, k, s, p)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, ss, idx, weight, mean, invstd = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        dev = x.device
        st = _lib.stream()
        dy = dy.contiguous(memory_format=torch.channels_last)
        dbn = torch.empty_like(x)
        w, b = ctx.params
        dg, db, direct = _param_grads(w, b, C, dev)
        slots, coef = _workspaces(C, dev)
        dx = torch.empty_like(x)
        if POOL_BN_STATS and C == 64 and k == 3 and s == 2:
            # pool gradient + the BN's backward statistics in one pass, then finalize + apply
            _lib.call("kfa_maxpool_bwd_bnstats", _lib.ptr(dy), _lib.ptr(idx), _lib.ptr(dbn), N, H, W, C, Ho, Wo, p,
                      _lib.ptr(x), _lib.ptr(ss), _lib.ptr(mean), _lib.ptr(slots), st)
            _lib.call("kfa_bn_bwd_prestats", _lib.ptr(dbn), _lib.ptr(x), None, _lib.ptr(weight), _lib.ptr(mean),
                      _lib.ptr(invstd), _lib.ptr(dx), None, _lib.ptr(dg), _lib.ptr(db), _lib.ptr(slots),
                      _lib.ptr(coef), N * H * W, C, 1, int(direct), _lib.ptr(ss), None, st)
        else:
            _lib.call("kfa_maxpool_bwd", _lib.ptr(dy), _lib.ptr(idx), _lib.ptr(dbn), N, H, W, C, Ho, Wo, k, s, p, st)
            _lib.call("kfa_bn_bwd", _lib.ptr(dbn), _lib.ptr(x), None, _lib.ptr(weight), _lib.ptr(mean),
                      _lib.ptr(invstd), _lib.ptr(dx), None, _lib.ptr(dg), _lib.ptr(db), _lib.ptr(slots),
                      _lib.ptr(coef), N * H * W, C, 1, int(direct), _lib.ptr(ss), None, st)
        if direct:
            notify_grad_ready(w)
            notify_grad_ready(b)
            return dx, None, None, None, None, None, None, None, None, None, None
        return (dx, dg if w.dtype == torch.float32 else dg.to(w.dtype), db if b.dtype == torch.float32 else db.to(b.dtype),
                None, None, None, None, None, None, None, None)


def bn_relu_maxpool(bn: "BatchNorm2dAct", x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1) -> torch.Tensor:
    """``max_pool2d(bn(x), k, s, p)`` for a BN with ReLU; fused in training on the
    GPU for the 3x3/s2 pool (:class:`_BNReluPoolFn`), else the two ops."""
    if (x.is_cuda and bn.training and bn.relu and MASK_FROM_X and k == 3 and s == 2 and p <= 1 and x.dim() == 4
            and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0):
        pre = getattr(x, "_kfa_prestats", False) and getattr(x, "_kfa_prestats_tag", "bn_slots") == "bn_slots"
        return _BNReluPoolFn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps, pre,
                                   k, s, p)
    from .pool import max_pool2d
    return max_pool2d(bn(x), k, s, p)


def bn_act_reference(x, weight, bias, running_mean, running_var, residual=None, training=True, momentum=0.1,
                     eps=1e-5, relu=True):
    """Plain PyTorch fp32 reference of the same op (used by the numerics tests)."""
    xf = x.float()
    y = torch.nn.functional.batch_norm(xf, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y


class BatchNorm2dAct(nn.Module):
    """``BatchNorm2d`` with an optional fused residual add and ReLU (NHWC bf16)."""

    def __init__(self, num_features: int, relu: bool = True, eps: float = 1e-5, momentum: float = 0.1,
                 zero_init: bool = False):
        super().__init__()
        self.num_features = num_features
        self.relu = relu
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.zeros(num_features) if zero_init else torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))

    def forward(self, x, residual=None, bwd_link: bool = False, res_join=None, lazy: bool = False):
        """``lazy``: the output feeds exactly one ``ops.conv.conv2d`` next, which folds the
        BN-apply + ReLU into its operand load where that measured faster (``LazyBN``)."""
        if x.is_cuda:
            pre = getattr(x, "_kfa_prestats", False) and getattr(x, "_kfa_prestats_tag", "bn_slots") == "bn_slots"
            return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, residual,
                          self.training, self.momentum, self.eps, self.relu, pre, bwd_link, res_join, lazy)
        # CPU path (plumbing tests / CPU-only MNIST-style jobs): plain PyTorch.
        y = torch.nn.functional.batch_norm(x, self.running_mean, self.running_var, self.weight.to(x.dtype),
                                           self.bias.to(x.dtype), self.training, self.momentum, self.eps)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if self.relu else y

    def extra_repr(self) -> str:
        return f"{self.num_features}, relu={self.relu}, eps={self.eps}, momentum={self.momentum}"
