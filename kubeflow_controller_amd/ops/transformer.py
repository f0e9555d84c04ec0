"""Transformer / recommender ops over the HIP kernels of ``csrc/kernels/transformer.hip``.

SURVEY §2.6 K1 (GEMM epilogues), K6 (embedding), K10 (LayerNorm), K11
(attention).  GEMMs are plain library GEMMs (``torch.mm``/``addmm``/``bmm`` →
hipBLASLt); everything around them is a hand-written kernel that fuses the
elementwise work (bias, activation, dropout, residual add, LayerNorm, head
split/merge, column-sum bias gradients) into one streaming pass.

The encoder layer is ONE autograd node (:class:`EncoderLayerFn`): backward is
written out explicitly so that

* weight gradients are accumulated straight into the flat gradient buffer
  (``gW.addmm_(dY.T, X)`` = hipBLASLt with beta=1) and bias / LayerNorm
  gradients are produced by the fused kernels into their flat views — the
  direct-gradient protocol of ``parallel/flat.py`` (no AccumulateGrad adds);
* the residual-gradient sums are folded into the dgrad GEMMs
  (``addmm(dres, dY, W)``), so no separate add kernel runs;
* dropout masks are regenerated from (seed, index) — never stored.

Every op has a plain-PyTorch fp32 reference (``*_reference``) used by the CPU
path and the numerics tests.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from . import gemm as _gemm
from . import streams as _streams
from . import loss as _loss  # noqa: F401  (registers kfa_softmax_xent)
from ..parallel.flat import direct_grad_view, notify_grad_ready

P, L, I, Fl = _lib.P, _lib.L, _lib.I, _lib.F
U64 = __import__("ctypes").c_ulonglong

_lib.register("kfa_ln_part_floats", [L, I], L)
_lib.register("kfa_colsum_part_floats", [L, I], L)
_lib.register("kfa_ln_fwd", [P, P, P, P, P, P, P, P, P, L, I, Fl, Fl, U64, P])
_lib.register("kfa_ln_bwd", [P, P, P, P, P, P, P, P, P, P, P, L, I, Fl, U64, I, P])
_lib.register("kfa_ln_bwd2", [P, P, P, P, P, P, P, P, P, P, P, P, L, I, Fl, U64, I, P])
_lib.register("kfa_bias_act_fwd", [P, P, P, L, I, I, Fl, U64, P])
_lib.register("kfa_bias_act_bwd", [P, P, P, P, P, P, L, I, I, Fl, U64, I, P])
_lib.register("kfa_scale_colsum", [P, P, P, L, I, P, I, P])
_lib.register("kfa_qkv_split", [P, P, P, P, P, L, I, I, I, Fl, P])
_lib.register("kfa_qkv_merge_bwd", [P, P, P, P, P, P, L, I, I, I, Fl, I, P])
_lib.register("kfa_heads_permute", [P, P, L, I, I, I, I, P])
_lib.register("kfa_attn_softmax_fwd", [P, P, P, L, I, I, Fl, U64, P])
_lib.register("kfa_attn_softmax_bwd", [P, P, L, I, Fl, U64, P])
_lib.register("kfa_embed_fwd", [P, P, P, P, P, P, I, P, L, I, L, P])
_lib.register("kfa_embed_bwd", [P, P, L, P, P, I, L, I, I, P])
_lib.register("kfa_colsum", [P, P, P, L, I, I, P])
_lib.register("kfa_embed_small_ws_floats", [I, I], restype=_lib.L)
_lib.register("kfa_embed_small_bwd", [P, P, _lib.L, P, I, _lib.L, I, I, P, P])
_lib.register("kfa_attn_fwd", [P, P, P, P, P, I, I, I, I, Fl, Fl, U64, P, P])
_lib.register("kfa_attn_bwd", [P, P, P, P, P, P, P, P, I, I, I, I, Fl, Fl, U64, P, P, P, P])
_lib.register("kfa_attn_dbias_part_floats", [I, I], L)
_lib.register("kfa_attn_mask_words", [I, I, I], _lib.L)

# env KFA_FUSED_ATTN=0 falls back to the split kernels + batched library GEMMs
FUSED_ATTN = os.environ.get("KFA_FUSED_ATTN", "1") != "0"

ACTS = {None: 0, "none": 0, "gelu": 1, "tanh": 2, "relu": 3}
SMALL_TABLE_ROWS = 1024
# tables of <= 8 rows (BERT's segment table): kfa_embed_small_bwd instead of the one-hot
# GEMM, whose M = R shape ran on hipBLASLt at ~140 us (KFA_EMB_SMALL=0 restores it)
EMB_SMALL_KERNEL = os.environ.get("KFA_EMB_SMALL", "1") != "0"
# KFA_FFN_GELU_EPI=1: the FFN-up forward also times the persistent GEMM with the bias +
# GELU epilogue (one launch instead of GEMM + pass).  Off by default: measured 0.299 ms vs
# 0.2255 for hipBLASLt + the bias/GELU pass (32768 x 3072 x 768) — its 8 stores per phase
# sit in the counted vmcnt window of the DMA retires and stall the pipeline.
FFN_GELU_EPI = os.environ.get("KFA_FFN_GELU_EPI", "0") == "1"
# KFA_DACT_EPI=1: the FFN-down data gradient through the GELU also times the
# wave-specialised GEMM with the GELU-backward epilogue (gemm_ppw_dact) against GEMM +
# bias_act_bwd.  Off by default: measured 392-425 vs 257-266 us (32768 x 3072 x 768) — the
# GELU' arithmetic (~25 VALU ops per element) lands on the store waves' share of the MFMA
# pipeline at the tile boundary, and the extra operand registers spill (docs/kernels.md).
DACT_EPI = os.environ.get("KFA_DACT_EPI", "0") == "1"
# KFA_ATTN_MASK=1: the encoder's attention forward stores its packed dropout keep mask
# and the backward reads it instead of re-hashing.  Off: the backward is HBM-bound
# once the hash is paired (BERT-base layer bwd 86 us re-hashing, 88 us without
# dropout, 96 us reading the mask — tools/bench_attn.py, docs/kernels.md).
ATTN_MASK = os.environ.get("KFA_ATTN_MASK", "0") == "1"
_MASK64 = (1 << 64) - 1


def mix_seed(*parts: int) -> int:
    """Deterministic 64-bit seed from integers (per layer / site / step)."""
    h = 0x243F6A8885A308D3
    for p in parts:
        h ^= (int(p) + 0x9E3779B97F4A7C15 + (h << 6) + (h >> 2)) & _MASK64
        h = (h * 0xBF58476D1CE4E5B9) & _MASK64
    return h


def s64(seed: int) -> int:
    """A 64-bit seed as the signed int64 with the same bits.  Seeds cross
    ``torch.autograd.Function.apply`` in this form: torch's profiler (record_shapes)
    converts Function arguments to int64 and rejects values >= 2^63.  Every consumer
    masks back to 64 bits (:func:`hash_key`, :func:`mix_seed`), so both forms give
    the same masks."""
    s = int(seed) & _MASK64
    return s - (1 << 64) if s >= (1 << 63) else s


def hash_key(seed: int) -> int:
    """The 64-bit key a kernel's dropout hash is launched with: ``seed`` mixed once
    per launch on the host.  ``drop_hash`` (``csrc/kernels/common.h``) folds its key
    into the element index linearly, so raw seeds that differ in a few bits (a
    step counter) would give index-permuted copies of one mask; mixed keys give
    unrelated masks.  Forward and backward launchers apply the same mapping."""
    return mix_seed(int(seed) & _MASK64, 0x5EED)


def _part(nfloats: int, device) -> torch.Tensor:
    return _lib.workspace(nfloats * 4, device, "colsum_part").view(torch.float32)


def _grad_target(p: torch.Tensor):
    """(buffer, accumulate, direct): the flat fp32/bf16 grad view when the param
    lives in a FlatGroup, else a fresh fp32 tensor returned through autograd."""
    v = direct_grad_view(p)
    if v is not None:
        return v, 1, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), 1, False


def _finish(p, buf, direct):
    if direct:  # the bucket launch joins the side stream (parallel/ddp.py, ps.py)
        notify_grad_ready(p)
        return None
    if buf.is_cuda:  # the weight gradient may still be in flight on the side stream
        _streams.join(buf.device)
    return buf.to(p.dtype)


# ----------------------------------------------------------------------------- raw launchers
def ln_fwd(x, gamma, beta, res=None, bias=None, eps=1e-12, p=0.0, seed=0, save_sum=True):
    rows, H = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty_like(x)
    xs = torch.empty_like(x) if save_sum and (res is not None or bias is not None or p > 0) else None
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty_like(mean)
    _lib.call("kfa_ln_fwd", _lib.ptr(x), _lib.ptr(res), _lib.ptr(bias), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(y),
              _lib.ptr(xs), _lib.ptr(mean), _lib.ptr(rstd), rows, H, eps, float(p), hash_key(seed), _lib.stream())
    return y, (xs if xs is not None else x), mean, rstd


def ln_bwd(dy, xs, mean, rstd, gamma, dgamma, dbeta, dbias=None, p=0.0, seed=0, want_branch=False, dy2=None):
    """LayerNorm backward of the gradient ``dy`` (+ ``dy2``, summed on the fly: a
    residual join whose projection dgrad then needs no addend)."""
    rows, H = dy.numel() // dy.shape[-1], dy.shape[-1]
    if dy2 is not None and (dy2.shape != dy.shape or dy2.dtype != dy.dtype or not dy2.is_contiguous()):
        raise ValueError(f"ln_bwd: dy2 {tuple(dy2.shape)} must match dy {tuple(dy.shape)}")
    dx = torch.empty_like(dy)
    dbr = torch.empty_like(dy) if (want_branch and p > 0) else None
    part = _part(_lib.lib().kfa_ln_part_floats(rows, H), dy.device)
    _lib.call("kfa_ln_bwd2", _lib.ptr(dy), _lib.ptr(dy2), _lib.ptr(xs), _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(gamma),
              _lib.ptr(dx), _lib.ptr(dbr), _lib.ptr(part), _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(dbias), rows, H,
              float(p), hash_key(seed), 1, _lib.stream())
    return dx, (dbr if dbr is not None else dx)


class ResidualJoin:
    """Gradient hand-off between consecutive encoder layers.  Layer L's input is
    layer L-1's output h, whose gradient is ``dx_res + dqkv · Wqkv`` (residual
    path + QKV-projection dgrad).  Layer L's backward deposits the projection
    term here and returns only ``dx_res``; layer L-1's backward takes it back and
    its LayerNorm backward sums the two on read (``ln_bwd(dy2=...)``).  So the
    dgrad is a plain GEMM (no addend epilogue, no beta = 1 read of C) and the sum
    is never written.  Only valid when h feeds nothing but layer L and the join
    consumer (``models/bert.py``); autograd's other consumers of h, if any, still
    add into ``dy`` as usual."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    def deposit(self, g: torch.Tensor) -> None:
        if self.g is not None:
            raise RuntimeError("ResidualJoin: gradient deposited twice (backward through the graph twice?)")
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


def bias_act_fwd(x, bias, act, p=0.0, seed=0):
    rows, N = x.numel() // x.shape[-1], x.shape[-1]
    y = torch.empty_like(x)
    _lib.call("kfa_bias_act_fwd", _lib.ptr(x), _lib.ptr(bias), _lib.ptr(y), rows, N, ACTS[act], float(p), hash_key(seed),
              _lib.stream())
    return y


def bias_act_bwd(dy, x, bias, act, dbias, p=0.0, seed=0, want_dx=True):
    rows, N = dy.numel() // dy.shape[-1], dy.shape[-1]
    dx = torch.empty_like(dy) if want_dx else None
    part = _part(_lib.lib().kfa_colsum_part_floats(rows, N), dy.device)
    _lib.call("kfa_bias_act_bwd", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(bias), _lib.ptr(dx), _lib.ptr(part),
              _lib.ptr(dbias), rows, N, ACTS[act], float(p), hash_key(seed), 1, _lib.stream())
    return dx


def colsum_(x, out):
    """out (+)= x.sum(0) over rows (fp32 out)."""
    rows, N = x.numel() // x.shape[-1], x.shape[-1]
    part = _part(_lib.lib().kfa_colsum_part_floats(rows, N), x.device)
    _lib.call("kfa_colsum", _lib.ptr(x), _lib.ptr(part), _lib.ptr(out), rows, N, 1, _lib.stream())


def _wgrad_(gw: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> None:
    """gW += dYᵀ·X straight into the flat grad view.

    The hand-written split-K MFMA wgrad kernel (``csrc/kernels/wgrad.hip``, the
    conv weight-gradient kernel run as a 1x1 conv over the token rows) beats
    hipBLASLt's transposed-A GEMM on these shapes (e.g. 16384x768x768: 374 vs
    215 TFLOP/s, ``tools/probe_wgrad_layouts.py``); hipBLASLt (``addmm_``,
    beta = 1) covers the shapes it does not take (dims not multiples of 8)."""
    from . import conv as _conv
    rows, out_f = dy2.shape
    in_f = x2.shape[1]
    if (_conv.WGRAD_ENABLED and gw.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and out_f % 8 == 0 and in_f % 8 == 0 and rows < (1 << 24) and gw.is_contiguous()
            and gw.dtype in (torch.bfloat16, torch.float32)):
        _conv.wgrad_into(x2.contiguous(), dy2.contiguous(), gw, 1, 1, rows, in_f, 1, rows, out_f, 1, 1, 1, 0,
                         accumulate=True)
        return
    if gw.dtype == dy2.dtype:
        gw.addmm_(dy2.t(), x2)
    else:
        gw.add_(torch.mm(dy2.t(), x2).to(gw.dtype))


def _wgrad_side_(gw: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> None:
    """:func:`_wgrad_` on the weight-gradient side stream (``ops/streams.py``):
    concurrent with the layer's data-gradient chain on the main stream."""
    if _streams.enabled(gw):
        _streams.run_on_side(lambda: _wgrad_(gw, dy2, x2), gw.device, (gw, dy2, x2))
    else:
        _wgrad_(gw, dy2, x2)


# ----------------------------------------------------------------------------- LayerNorm
class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        x = x.contiguous()
        y, xs, mean, rstd = ln_fwd(x, gamma, beta, eps=eps)
        ctx.save_for_backward(xs, mean, rstd, gamma)
        ctx.params = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, mean, rstd, gamma = ctx.saved_tensors
        g, b = ctx.params
        gg, _, dg = _grad_target(g)
        gb, _, db = _grad_target(b)
        dx, _ = ln_bwd(dy.contiguous(), xs, mean, rstd, gamma, gg, gb)
        return dx, _finish(g, gg, dg), _finish(b, gb, db), None


def layer_norm(x, gamma, beta, eps=1e-12):
    if not x.is_cuda:
        return F.layer_norm(x, (x.shape[-1],), gamma.to(x.dtype), beta.to(x.dtype), eps)
    return LayerNormFn.apply(x, gamma, beta, eps)


# ----------------------------------------------------------------------------- dense + bias + act
class DenseFn(torch.autograd.Function):
    """y = dropout(act(x · Wᵀ + b)).

    Without dropout the whole layer is ONE launch of the MFMA GEMM with the
    bias / activation epilogue (``ops/gemm.py``), which also keeps the
    pre-activation for the backward; the dgrad runs on the same kernel against
    the transposed weight.  With dropout: library GEMM + one fused epilogue pass."""

    @staticmethod
    def forward(ctx, x, weight, bias, act, p, seed):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        has_act = act not in (None, "none")
        fusable = p == 0 and _gemm.gemm_ok(x2, weight) and (
            bias is None or (bias.dtype == torch.float32 and bias.is_contiguous() and bias.data_ptr() % 16 == 0))
        fused = fusable and (_gemm.ROUTE_LAYERS or (_gemm.ROUTE_FUSED and has_act))
        _gemm.mark_weights_stale()  # the dgrad's cached weight transposes refresh at the next backward
        mm = None  # plain GEMM of the unfused path (None: hipBLASLt)
        skinny = None  # split count of the split-K skinny GEMM with the bias fused (M <= 256, e.g. the ResNet FC)
        relu_y = False  # the persistent GEMM with the bias + ReLU epilogue: y only, the backward masks by y > 0
        if fusable and _gemm.ROUTE_AUTO:
            # per shape, the fastest of: hipBLASLt + one bias/act pass, the MFMA GEMM with
            # the bias/act epilogue fused, the persistent MFMA GEMM + the bias/act pass,
            # the skinny split-K GEMM with the bias fused (+ the act pass)
            ba = (lambda zz: bias_act_fwd(zz, bias, act) if (bias is not None or has_act) else zz)  # noqa: E731
            act_only = (lambda zz: bias_act_fwd(zz, None, act) if has_act else zz)  # noqa: E731
            own_pp = _gemm._ppp_candidates(x2, weight) if _gemm.ppp_ok(x2, weight) else []
            cands = ([("hipblaslt", lambda: ba(torch.mm(x2, weight.t()))),
                      ("gemm_nt-fused", lambda: _gemm.gemm_nt(x2, weight, bias=bias, act=act, want_z=has_act))]
                     + [(n, (lambda f: lambda: ba(f()))(f)) for n, f in own_pp])
            relu_fns = []  # bias + ReLU epilogue variants: y only, the backward masks by y > 0
            if act == "relu" and own_pp and _gemm.ppp_gelu_ok(x2, weight, bias):
                relu_fns = [("ppp256-relu", lambda: _gemm.gemm_ppp_relu(x2, weight, bias)),
                            ("ppw256-relu", lambda: _gemm.gemm_ppw_relu(x2, weight, bias)),
                            ("ppw256-nt-relu", lambda: _gemm.gemm_ppw_relu(x2, weight, bias, nt=True))]
                cands += relu_fns
            sk = _gemm.skinny_splits(x2, weight) if _gemm.skinny_ok(x2, weight) else []
            cands += [(n + "-bias", (lambda s: lambda: act_only(_gemm.gemm_skinny(x2, weight, bias, splits=s)))(s))
                      for n, s in sk]
            i = _gemm.pick_fastest("dense_fwd", (x2.shape[0], weight.shape[0], x2.shape[1], act, bias is not None),
                                   x2.device, cands)
            fused = i == 1
            ns = len(cands) - len(sk)
            skinny = sk[i - ns][1] if i >= ns else None
            mm = own_pp[i - 2][1] if 2 <= i < 2 + len(own_pp) else None
            r0 = 2 + len(own_pp)
            relu_y = relu_fns[i - r0][1] if r0 <= i < r0 + len(relu_fns) else False
        if fused:
            y, z = _gemm.gemm_nt(x2, weight, bias=bias, act=act, want_z=has_act)  # z includes the bias
        elif relu_y:
            y = relu_y()
            z = y  # relu'(z + b) == (y > 0): the output stands in for the pre-activation
        elif skinny is not None:
            z = _gemm.gemm_skinny(x2, weight, bias, splits=skinny)  # z includes the bias
            y = bias_act_fwd(z, None, act, p, seed) if (has_act or p > 0) else z
        else:
            z = mm() if mm is not None else torch.mm(x2, weight.t())
            y = bias_act_fwd(z, bias, act, p, seed) if (bias is not None or has_act or p > 0) else z
        ctx.save_for_backward(x2, weight, z if has_act else None)
        ctx.bias = bias
        ctx.cfg = (act, p, seed, shp, fused, fused or skinny is not None or bool(relu_y))
        return y.view(*shp[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, z = ctx.saved_tensors
        bias = ctx.bias
        act, p, seed, shp, fused, z_has_bias = ctx.cfg
        has_act = act not in (None, "none")
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        gb = db = None
        if bias is not None:
            gb, _, db = _grad_target(bias)
        if has_act or p > 0 or bias is not None:
            # fused forward: z already holds the bias, so act' is evaluated at z itself
            dz = bias_act_bwd(dy2, z, None if z_has_bias else bias, act, gb, p, seed, want_dx=(has_act or p > 0))
            dz = dy2 if dz is None else dz
        else:
            dz = dy2
        dx = None
        if ctx.needs_input_grad[0]:
            own_dx = fused and _gemm.ROUTE_LAYERS and weight.shape[1] % 8 == 0
            wt = _gemm.transpose(weight) if own_dx else None
            if wt is not None and _gemm.gemm_ok(dz, wt):
                dx = _gemm.gemm_nt(dz, wt)[0].view(shp)
            else:  # per shape: the persistent MFMA GEMM on the transposed weight, or hipBLASLt
                dx = _gemm.dgrad_auto(dz, weight, "dense_dgrad").view(shp)
        gw, _, dw = _grad_target(weight)
        _wgrad_(gw, dz, x2)
        return dx, _finish(weight, gw, dw), (_finish(bias, gb, db) if bias is not None else None), None, None, None


def dense(x, weight, bias=None, act=None, p=0.0, seed=0):
    if not x.is_cuda:
        return dense_reference(x, weight, bias, act)
    return DenseFn.apply(x, weight, bias, act, float(p), s64(seed))


def _act_ref(z, act):
    if act == "gelu":
        return F.gelu(z)
    if act == "tanh":
        return torch.tanh(z)
    if act == "relu":
        return torch.relu(z)
    return z


def dense_reference(x, weight, bias=None, act=None):
    z = x @ weight.to(x.dtype).t()
    if bias is not None:
        z = z + bias.to(z.dtype)
    return _act_ref(z, act)


# ----------------------------------------------------------------------------- embeddings
class EmbeddingSumFn(torch.autograd.Function):
    """out[r] = Σ_k table_k[ids_k[r]] (≤ 3 tables); sparse backward through a
    self-cleaning fp32 scratch per table (touches only the looked-up rows)."""

    @staticmethod
    def forward(ctx, ids0, ids1, ids2, t0, t1, t2):
        tabs = [t0, t1, t2]
        ids = [ids0, ids1, ids2]
        D = t0.shape[1]
        n = ids0.numel()
        out = torch.empty(n, D, dtype=torch.bfloat16, device=t0.device)
        f32 = sum(1 << k for k, t in enumerate(tabs) if t is not None and t.dtype == torch.float32)
        ids = [i.reshape(-1).contiguous() if i is not None else None for i in ids]
        _lib.call("kfa_embed_fwd", _lib.ptr(ids[0]), _lib.ptr(t0), _lib.ptr(ids[1]), _lib.ptr(t1), _lib.ptr(ids[2]),
                  _lib.ptr(t2), f32, _lib.ptr(out), n, D, D, _lib.stream())
        ctx.save_for_backward(*[i if i is not None else torch.empty(0) for i in ids])
        ctx.tabs = tabs
        return out.view(*ids0.shape, D)

    @staticmethod
    def backward(ctx, dout):
        ids = ctx.saved_tensors
        dout = dout.reshape(-1, dout.shape[-1]).contiguous()
        n, D = dout.shape
        grads = []
        for k, t in enumerate(ctx.tabs):
            if t is None or not ctx.needs_input_grad[3 + k]:
                grads.append(None)
                continue
            g, _, direct = _grad_target(t)
            if (EMB_SMALL_KERNEL and t.shape[0] <= 8 and D % 8 == 0 and g.dtype in (torch.float32, torch.bfloat16)
                    and g.is_contiguous() and ids[k].dtype == torch.int64):
                # per-chunk LDS images of the table's gradient, summed in chunk order into g
                R = t.shape[0]
                part = _lib.workspace(4 * _lib.lib().kfa_embed_small_ws_floats(R, D), t.device, "embed_small_part")
                _lib.call("kfa_embed_small_bwd", _lib.ptr(ids[k]), _lib.ptr(dout), D, _lib.ptr(g),
                          int(g.dtype == torch.float32), n, D, R, _lib.ptr(part), _lib.stream())
            elif t.shape[0] <= SMALL_TABLE_ROWS:
                # few rows, many duplicates (position / segment tables): atomics would
                # serialise on a handful of addresses; a one-hot GEMM (MFMA) reduces them
                oh = torch.zeros(n, t.shape[0], dtype=dout.dtype, device=dout.device)
                oh.scatter_(1, ids[k].view(-1, 1), 1.0)
                _wgrad_(g, oh, dout)
            else:
                scratch = _lib.workspace(t.shape[0] * D * 4, t.device, f"embed_scratch{k}").view(torch.float32)
                _lib.call("kfa_embed_bwd", _lib.ptr(ids[k]), _lib.ptr(dout), D, _lib.ptr(scratch), _lib.ptr(g),
                          int(g.dtype == torch.float32), n, D, 1, _lib.stream())
            grads.append(_finish(t, g, direct))
        return (None, None, None, *grads)


def embedding_sum(tables, ids):
    """Σ_k tables[k][ids[k]] as bf16 ``[*ids[0].shape, D]``."""
    tables = list(tables) + [None] * (3 - len(tables))
    ids = list(ids) + [None] * (3 - len(ids))
    if not tables[0].is_cuda:
        out = 0
        for t, i in zip(tables, ids):
            if t is not None:
                out = out + F.embedding(i, t.float())
        return out
    return EmbeddingSumFn.apply(ids[0], ids[1], ids[2], tables[0], tables[1], tables[2])


# ----------------------------------------------------------------------------- fused attention
def fused_attention_ok(S: int, d: int) -> bool:
    """``csrc/kernels/attention.hip`` covers head dim 64 at S = 128 (one workgroup per
    head) and S = 128·n up to 8192 (128-query blocks, online softmax; BERT phase 2: 512)."""
    return FUSED_ATTN and S % 128 == 0 and 0 < S <= 8192 and d == 64


def _attn_biases(bqkv, key_bias, W3, T_, dev):
    """The kernels always read both biases (no branches around their prologue
    loads): absent ones become zeros."""
    if bqkv is None:
        bqkv = _zeros_f32(W3, dev)
    elif bqkv.dtype != torch.float32 or bqkv.numel() != W3 or not bqkv.is_contiguous():
        raise ValueError("attention: bqkv must be a contiguous fp32 [3H] vector")
    if key_bias is None:  # no padding mask: one cached zero vector, not a fill kernel per call
        key_bias = _zeros_f32(T_, dev)
    return bqkv, key_bias


def _zeros_f32(n: int, dev) -> torch.Tensor:
    """A read-only fp32 zero vector of ``n`` elements (grow-only workspace that no kernel
    writes: the zero-initialised buffer stays zero)."""
    return _lib.workspace(4 * n, dev, "const_zeros_f32").view(torch.float32)[:n]


def attn_fwd(qkv, bqkv, key_bias, B, S, heads, p=0.0, seed=0, want_mask=False):
    """(ctx [B*S, H], lse [B*heads, S]) of softmax((q+b)(k+b)ᵀ/√d + key_bias)·(v+b), dropout p.

    ``want_mask``: also return the packed dropout keep mask the S = 128 kernel
    writes (int32 [B*heads, 4, S], 2 KiB per head; None when there is no dropout or
    another kernel runs) — :func:`attn_bwd` reads it instead of re-hashing every
    score.  Dropout: one counter hash per score pair, 16-bit thresholds
    (``csrc/kernels/attention.hip``: attn_pair_hash)."""
    T_, W3 = qkv.shape
    H = W3 // 3
    d = H // heads
    if not (fused_attention_ok(S, d) and T_ == B * S and qkv.is_contiguous() and qkv.dtype == torch.bfloat16):
        raise ValueError(f"attn_fwd: unsupported shape qkv {tuple(qkv.shape)}, B={B} S={S} heads={heads}")
    if key_bias is not None and (key_bias.dtype != torch.float32 or key_bias.numel() != B * S
                                 or not key_bias.is_contiguous()):
        raise ValueError("attn_fwd: key_bias must be a contiguous fp32 [B, S] tensor")
    bqkv, key_bias = _attn_biases(bqkv, key_bias, W3, B * S, qkv.device)
    out = torch.empty(T_, H, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(B * heads, S, dtype=torch.float32, device=qkv.device)
    mask = None
    if want_mask and p > 0:
        words = _lib.lib().kfa_attn_mask_words(B, S, heads)
        if words:
            mask = torch.empty(B * heads, 4, S, dtype=torch.int32, device=qkv.device)
            assert mask.numel() == words
    _lib.call("kfa_attn_fwd", _lib.ptr(qkv), _lib.ptr(bqkv), _lib.ptr(key_bias), _lib.ptr(out), _lib.ptr(lse), B, S,
              heads, d, 1.0 / math.sqrt(d), float(p), hash_key(seed), _lib.ptr(mask), _lib.stream())
    return (out, lse, mask) if want_mask else (out, lse)


def attn_bwd(qkv, bqkv, key_bias, out, lse, dout, dbqkv, B, S, heads, p=0.0, seed=0, mask=None):
    """dqkv [B*S, 3H] of :func:`attn_fwd` (``out``, ``lse``, ``mask``: its outputs); the
    bias gradient is added into ``dbqkv`` (fp32, nullable).  Without ``mask`` the
    kernel regenerates the dropout decisions from the hash (same values)."""
    T_, W3 = qkv.shape
    H = W3 // 3
    d = H // heads
    dout = dout.contiguous()
    if tuple(dout.shape) != (T_, H) or dout.dtype != qkv.dtype:
        raise ValueError("attn_bwd: dout must be bf16 [B*S, H]")
    if tuple(out.shape) != (T_, H) or out.dtype != qkv.dtype or not out.is_contiguous():
        raise ValueError("attn_bwd: out must be the contiguous bf16 [B*S, H] forward output")
    bqkv, key_bias = _attn_biases(bqkv, key_bias, W3, B * S, qkv.device)
    if mask is not None and (mask.dtype != torch.int32 or mask.numel() != _lib.lib().kfa_attn_mask_words(B, S, heads)
                             or not mask.is_contiguous()):
        raise ValueError("attn_bwd: mask must be the forward's int32 [B*heads, 4, S] keep mask")
    dqkv = torch.empty_like(qkv)
    work = _lib.workspace(B * heads * S * 4, qkv.device, "attn_rowdot")  # D = rowsum(dO∘O) (S > 128)
    # the S = 128 kernel's bias gradient: per-(sequence, wave) partial rows, then one sum
    dbpart = (_lib.workspace(_lib.lib().kfa_attn_dbias_part_floats(B, heads) * 4, qkv.device, "attn_dbias")
              if dbqkv is not None else None)
    _lib.call("kfa_attn_bwd", _lib.ptr(qkv), _lib.ptr(bqkv), _lib.ptr(key_bias), _lib.ptr(out), _lib.ptr(lse),
              _lib.ptr(dout), _lib.ptr(dqkv), _lib.ptr(dbqkv), B, S, heads, d, 1.0 / math.sqrt(d), float(p),
              hash_key(seed), _lib.ptr(mask if p > 0 else None), _lib.ptr(work), _lib.ptr(dbpart), _lib.stream())
    return dqkv


def _ffn_up(h, w, b):
    """FFN-up forward ``(gelu(h @ w.T + b), z, z_has_bias)``: per shape the fastest of
    the GEMM (hipBLASLt or an own persistent variant) + the bias/GELU pass, and the own
    persistent GEMM with the bias + GELU epilogue (one launch, ``gemm_ppp_gelu``)."""
    if _gemm.ROUTE_AUTO and FFN_GELU_EPI and _gemm.ppp_gelu_ok(h, w, b):
        own_pp = _gemm._ppp_candidates(h, w)
        cands = ([("hipblaslt+pass", lambda: bias_act_fwd(torch.mm(h, w.t()), b, "gelu"))]
                 + [(n + "+pass", (lambda f: lambda: bias_act_fwd(f(), b, "gelu"))(f)) for n, f in own_pp]
                 + [("ppp256-gelu", lambda: _gemm.gemm_ppp_gelu(h, w, b))])
        i = _gemm.pick_fastest("ffn_up", (h.shape[0], w.shape[0], h.shape[1]), h.device, cands)
        if i == len(cands) - 1:
            y, z = _gemm.gemm_ppp_gelu(h, w, b)
            return y, z, True
        z = own_pp[i - 1][1]() if i > 0 else torch.mm(h, w.t())
        return bias_act_fwd(z, b, "gelu"), z, False
    z = _gemm.mm_auto(h, w)
    return bias_act_fwd(z, b, "gelu"), z, False


def _ffn_down_dgrad_gelu(df2, w2, z, bias, dbias):
    """``dz = (df2 @ w2) * gelu'(z + bias)`` and ``dbias += colsum(dz)`` — the FFN-down
    data gradient through the GELU: per shape the faster of the data-gradient GEMM
    (:func:`ops.gemm.dgrad_auto`) + the ``bias_act_bwd`` pass, and the wave-specialised
    persistent GEMM with the GELU-backward epilogue (``gemm_ppw_dact``: one GEMM
    launch, no 3-tensor pass).  The timing runs accumulate into a scratch bias gradient."""
    if _gemm.ROUTE_AUTO and DACT_EPI and df2.is_cuda:
        w2t = _gemm.transpose_cached(w2)
        if _gemm.ppw_dact_ok(df2, w2t, z) and dbias is not None and dbias.dtype == torch.float32:
            key = (df2.shape[0], w2.shape[1], df2.shape[1])
            hit = _gemm._choice.get(("ffn_down_dgelu",) + key)
            if hit is None:
                scratch = torch.zeros_like(dbias)
                cands = [("dgrad+pass", lambda: bias_act_bwd(_gemm.dgrad_auto(df2, w2), z, bias, "gelu", scratch)),
                         ("ppw-dact", lambda: _gemm.gemm_ppw_dact(df2, w2t, z, bias, scratch)),
                         ("ppw-dact-nt", lambda: _gemm.gemm_ppw_dact(df2, w2t, z, bias, scratch, nt=True))]
                hit = _gemm.pick_fastest("ffn_down_dgelu", key, df2.device, cands)
            if hit:
                return _gemm.gemm_ppw_dact(df2, w2t, z, bias, dbias, nt=hit == 2)
    return bias_act_bwd(_gemm.dgrad_auto(df2, w2), z, bias, "gelu", dbias)


# ----------------------------------------------------------------------------- encoder layer
class EncoderLayerFn(torch.autograd.Function):
    """Post-LN BERT encoder layer, forward + backward written out (see module doc).

    Inputs: x [T, H] bf16 (T = B·S), key_bias [B, S] fp32 additive mask (or None),
    then the 12 parameters.  cfg = (B, S, heads, p_hidden, p_attn, seed, eps).

    MI355X path: the four projections (forward and dgrad) run on the MFMA GEMM of
    ``ops/gemm.py`` — FFN-up with its bias + GELU epilogue (keeping the
    pre-activation), its dgrad with the GELU backward + bias-gradient column sums
    fused in, the residual-gradient joins as GEMM addends — and attention is ONE
    fused kernel each way (``csrc/kernels/attention.hip``, S = 128, d = 64) that
    reads the QKV projection and writes the context / the QKV gradient directly.
    Other shapes fall back to library GEMMs + the split attention kernels."""

    @staticmethod
    def forward(ctx, x, key_bias, cfg, wqkv, bqkv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2):
        # cfg[7:9] (optional): ResidualJoin of this layer's input (deposited into by
        # the backward) and of its output (taken from by the backward)
        B, S, heads, ph, pa, seed, eps = cfg[:7]
        ctx.joins = (tuple(cfg[7:9]) + (None, None))[:2]
        _gemm.mark_weights_stale()  # the dgrad's cached weight transposes refresh at the next backward
        T, H = x.shape
        d = H // heads
        qscale = 1.0 / math.sqrt(d)
        st = _lib.stream()
        dev = x.device
        s_attn, s_h1, s_h2 = mix_seed(seed, 1), mix_seed(seed, 2), mix_seed(seed, 3)
        use_g = _gemm.ROUTE_LAYERS and _gemm.gemm_ok(x, wqkv) and _gemm.gemm_ok(x, w1) and w2.shape[0] % 8 == 0 and w2.shape[1] % 8 == 0
        use_f = use_g or (_gemm.ROUTE_FUSED and _gemm.gemm_ok(x, w1) and w2.shape[0] % 8 == 0 and w2.shape[1] % 8 == 0)
        # plain projections: the fused-epilogue MFMA GEMM (KFA_GEMM=1), else per shape the
        # persistent MFMA GEMM or hipBLASLt, whichever measured faster (ops/gemm.mm_auto)
        mm = (lambda a, w: _gemm.gemm_nt(a, w)[0]) if use_g else _gemm.mm_auto  # noqa: E731
        fused = fused_attention_ok(S, d)
        # attention
        qkv = mm(x, wqkv)                                                 # [T, 3H]
        if fused:
            ctxr, lse, amask = attn_fwd(qkv, bqkv, key_bias, B, S, heads, pa, s_attn, want_mask=True) if ATTN_MASK \
                else attn_fwd(qkv, bqkv, key_bias, B, S, heads, pa, s_attn) + (None,)
            att = (qkv, lse, amask)
        else:
            q = torch.empty(B * heads, S, d, dtype=x.dtype, device=dev)
            k = torch.empty_like(q)
            v = torch.empty_like(q)
            _lib.call("kfa_qkv_split", _lib.ptr(qkv), _lib.ptr(bqkv), _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), T, S,
                      heads, d, qscale, st)
            del qkv
            probs = torch.bmm(q, k.transpose(1, 2))                       # [BH, S, S]
            pdrop = torch.empty_like(probs) if pa > 0 else None
            _lib.call("kfa_attn_softmax_fwd", _lib.ptr(probs), _lib.ptr(key_bias), _lib.ptr(pdrop), B * heads * S,
                      S, heads, float(pa), s_attn, st)
            ctx_h = torch.bmm(pdrop if pdrop is not None else probs, v)    # [BH, S, d]
            ctxr = torch.empty(T, H, dtype=x.dtype, device=dev)
            _lib.call("kfa_heads_permute", _lib.ptr(ctx_h), _lib.ptr(ctxr), T, S, heads, d, 1, st)
            del ctx_h
            att = (q, k, v, probs, pdrop)
        ao = mm(ctxr, wo)
        h1, h1s, m1, r1 = ln_fwd(ao, g1, be1, res=x, bias=bo, eps=eps, p=ph, seed=s_h1)
        del ao
        # feed-forward; f1 = pre-activation (GEMM path: bias included)
        z_bias = use_f  # f1 includes b1 (the backward's GELU' then takes no bias)
        if use_f:
            f1a, f1 = _gemm.gemm_nt(h1, w1, bias=b1, act="gelu", want_z=True)
        else:
            f1a, f1, z_bias = _ffn_up(h1, w1, b1)
        f2 = mm(f1a, w2)
        h2, h2s, m2, r2 = ln_fwd(f2, g2, be2, res=h1, bias=b2, eps=eps, p=ph, seed=s_h2)
        ctx.save_for_backward(x, ctxr, h1, h1s, m1, r1, f1, f1a, h2s, m2, r2, *att)
        ctx.params = (wqkv, bqkv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2)
        ctx.cfg = (B, S, heads, ph, pa, (s_attn, s_h1, s_h2), qscale, use_g, use_f, fused, z_bias)
        ctx.key_bias = key_bias
        return h2

    @staticmethod
    def backward(ctx, dy):
        (x, ctxr, h1, h1s, m1, r1, f1, f1a, h2s, m2, r2, *att) = ctx.saved_tensors
        wqkv, bqkv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2 = ctx.params
        B, S, heads, ph, pa, (s_attn, s_h1, s_h2), qscale, use_g, use_f, fused, z_bias = ctx.cfg
        key_bias = ctx.key_bias
        T, H = x.shape
        d = H // heads
        st = _lib.stream()
        dy = dy.contiguous()
        join_in, join_out = ctx.joins
        tg = {id(p): _grad_target(p) for p in ctx.params}
        G = lambda p: tg[id(p)][0]  # noqa: E731
        # LN2 (+ FFN2 bias grad, hidden dropout): dres -> h1, dbranch -> f2; the next
        # layer's QKV dgrad (its ResidualJoin deposit) is summed in on read
        dy2 = join_out.take() if join_out is not None else None
        dh1_res, df2 = ln_bwd(dy, h2s, m2, r2, g2, G(g2), G(be2), G(b2), p=ph, seed=s_h2, want_branch=True, dy2=dy2)
        del dy2
        _wgrad_side_(G(w2), df2, f1a)
        if use_f:   # df1 = (df2 · W2) * gelu'(z1), db1 += colsum(df1): one GEMM launch
            df1 = _gemm.gemm_nt(df2, _gemm.transpose(w2), zin=f1, dact="gelu", dbias=G(b1))[0]
        else:
            df1 = _ffn_down_dgrad_gelu(df2, w2, f1, None if z_bias else b1, G(b1))
        del df2
        _wgrad_side_(G(w1), df1, h1)
        if use_g:   # residual-gradient join as the GEMM addend
            dh1, dh1b = _gemm.gemm_nt(df1, _gemm.transpose(w1), addend=dh1_res)[0], None
        else:       # plain dgrad; LN1's backward sums the residual gradient on read
            dh1, dh1b = dh1_res, _gemm.dgrad_auto(df1, w1)
        del df1, dh1_res
        # LN1 (+ out-proj bias grad)
        dx_res, dao = ln_bwd(dh1, h1s, m1, r1, g1, G(g1), G(be1), G(bo), p=ph, seed=s_h1, want_branch=True, dy2=dh1b)
        del dh1, dh1b
        _wgrad_side_(G(wo), dao, ctxr)
        dctxr = _gemm.gemm_nt(dao, _gemm.transpose(wo))[0] if use_g else _gemm.dgrad_auto(dao, wo)
        res_shared = dao is dx_res  # no hidden dropout: one tensor, also the side stream's wgrad operand
        del dao
        if fused:
            qkv, lse, amask = att
            # QKV-bias gradient: a column-sum pass over dqkv (it is still in the Infinity
            # Cache); KFA_ATTN_DBIAS=1: the kernel's per-(sequence, wave) column sums of the
            # tile it stores (partial rows + one small sum) — +10 us in the kernel, no net gain
            if ATTN_DBIAS:
                dqkv = attn_bwd(qkv, bqkv, key_bias, ctxr, lse, dctxr, G(bqkv), B, S, heads, pa, s_attn, mask=amask)
            else:
                dqkv = attn_bwd(qkv, bqkv, key_bias, ctxr, lse, dctxr, None, B, S, heads, pa, s_attn, mask=amask)
                colsum_(dqkv, G(bqkv))
            del dctxr
        else:
            q, k, v, probs, pdrop = att
            dctx_h = torch.empty(B * heads, S, d, dtype=dy.dtype, device=dy.device)
            _lib.call("kfa_heads_permute", _lib.ptr(dctxr), _lib.ptr(dctx_h), T, S, heads, d, 0, st)
            del dctxr
            pd = pdrop if pdrop is not None else probs
            dv = torch.bmm(pd.transpose(1, 2), dctx_h)
            dp = torch.bmm(dctx_h, v.transpose(1, 2))
            del dctx_h
            _lib.call("kfa_attn_softmax_bwd", _lib.ptr(probs), _lib.ptr(dp), B * heads * S, S, float(pa), s_attn, st)
            dq = torch.bmm(dp, k)
            dk = torch.bmm(dp.transpose(1, 2), q)
            del dp
            dqkv = torch.empty(T, 3 * H, dtype=dy.dtype, device=dy.device)
            W3 = 3 * H
            part = _part(_lib.lib().kfa_colsum_part_floats(T, W3), dy.device)
            _lib.call("kfa_qkv_merge_bwd", _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv), _lib.ptr(dqkv), _lib.ptr(part),
                      _lib.ptr(G(bqkv)), T, S, heads, d, qscale, 1, st)
            del dq, dk, dv
        _wgrad_side_(G(wqkv), dqkv, x)
        if use_g:
            dx = _gemm.gemm_nt(dqkv, _gemm.transpose(wqkv), addend=dx_res)[0]
        elif join_in is not None:  # the previous layer's LN2 backward adds it on read
            join_in.deposit(_gemm.dgrad_auto(dqkv, wqkv))
            dx = dx_res
        elif res_shared:  # never written in place while the side stream may read it
            dx = torch.addmm(dx_res, dqkv, wqkv)
        else:
            dx = dx_res.addmm_(dqkv, wqkv)
        grads = [_finish(p, tg[id(p)][0], tg[id(p)][2]) for p in ctx.params]
        return (dx, None, None, *grads)


def encoder_layer_reference(x, key_bias, cfg, wqkv, bqkv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2):
    """Plain PyTorch fp32 reference (no dropout)."""
    B, S, heads, _, _, _, eps = cfg
    T, H = x.shape
    d = H // heads
    f = lambda t: t.float()  # noqa: E731
    x = f(x)
    qkv = x @ f(wqkv).t() + f(bqkv)
    q, k, v = qkv.view(B, S, 3, heads, d).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2)) / math.sqrt(d)
    if key_bias is not None:
        sc = sc + key_bias.view(B, 1, 1, S)
    a = torch.softmax(sc, -1) @ v
    a = a.permute(0, 2, 1, 3).reshape(T, H)
    h1 = F.layer_norm(a @ f(wo).t() + f(bo) + x, (H,), f(g1), f(be1), eps)
    ff = F.gelu(h1 @ f(w1).t() + f(b1)) @ f(w2).t() + f(b2)
    return F.layer_norm(ff + h1, (H,), f(g2), f(be2), eps)


# ----------------------------------------------------------------------------- dropout / decoder + loss
class DropoutFn(torch.autograd.Function):
    """Counter-hash dropout (mask regenerated in backward from the seed)."""

    @staticmethod
    def forward(ctx, x, p, seed):
        x = x.contiguous()
        ctx.cfg = (p, seed)
        return bias_act_fwd(x, None, None, p, seed)

    @staticmethod
    def backward(ctx, dy):
        p, seed = ctx.cfg
        return bias_act_bwd(dy.contiguous(), None, None, None, None, p, seed), None, None


def dense_dropout(x, p, seed):
    if p <= 0:
        return x
    if not x.is_cuda:
        return F.dropout(x, p)
    return DropoutFn.apply(x, float(p), s64(seed))


DEC_SCALE_COLSUM = os.environ.get("KFA_DEC_SCALE_COLSUM", "1") != "0"
ATTN_DBIAS = os.environ.get("KFA_ATTN_DBIAS", "0") == "1"  # measured equal / slower than the pass (docs/kernels.md)


class DecoderXentFn(torch.autograd.Function):
    """mean softmax-xent of ``t · Wᵀ + b`` (tied MLM decoder): the bias is added
    inside the loss kernel and dlogits is produced in the forward pass."""

    @staticmethod
    def forward(ctx, t, w, b, labels):
        t = t.contiguous()
        logits = _gemm.mm_auto(t, w, "decoder")
        n, V = logits.shape
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        row_loss = torch.empty(n, dtype=torch.float32, device=t.device)
        dlog = torch.empty_like(logits)
        _lib.call("kfa_softmax_xent", _lib.ptr(logits), 1, _lib.ptr(lab), _lib.ptr(b), _lib.ptr(row_loss),
                  _lib.ptr(dlog), n, V, 1.0 / n, 0.0, _lib.stream())
        del logits
        ctx.save_for_backward(t, w, dlog)
        ctx.params = (w, b)
        return row_loss.sum() / n

    @staticmethod
    def backward(ctx, g):
        t, w, dlog = ctx.saved_tensors
        wp, bp = ctx.params
        # dlogits * g and the decoder-bias gradient in one pass over the logits-sized
        # tensor (g stays on the device: no host sync)
        n, V = dlog.shape
        gb, _, db = _grad_target(bp)
        if not DEC_SCALE_COLSUM:  # A/B: torch mul_ + a separate column-sum pass
            dlog.mul_(g.to(dlog.dtype))
            dt = _gemm.dgrad_auto(dlog, w, "decoder_dgrad")
            gw, _, dw = _grad_target(wp)
            _wgrad_(gw, dlog, t)
            colsum_(dlog, gb)
            return dt, _finish(wp, gw, dw), _finish(bp, gb, db), None
        gs = g.detach().to(torch.float32).reshape(1).contiguous()
        dls = torch.empty_like(dlog)
        _lib.call("kfa_scale_colsum", _lib.ptr(dlog), _lib.ptr(dls), _lib.ptr(gb), n, V, _lib.ptr(gs), 1, _lib.stream())
        del dlog
        dt = _gemm.dgrad_auto(dls, w, "decoder_dgrad")
        gw, _, dw = _grad_target(wp)
        _wgrad_(gw, dls, t)
        return dt, _finish(wp, gw, dw), _finish(bp, gb, db), None


def decoder_xent(t, w, b, labels):
    return DecoderXentFn.apply(t, w, b, labels)
