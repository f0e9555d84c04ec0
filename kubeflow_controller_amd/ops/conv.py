"""NHWC bf16 2-D convolution on the hand-written MFMA implicit GEMM
(``csrc/kernels/conv_igemm.hip``) — SURVEY §2.6 K7.

* forward: implicit GEMM over the NHWC input (``sa = stride, ra = +1, oa = -pad``);
* dgrad, stride 1: implicit GEMM over dY with flipped taps (``ra = -1, oa = +pad``)
  against the weight transposed to ``[Cin][R][S][Cout]``;
* dgrad, stride 2: split by output parity class (ph, pw); each class is a
  stride-1 implicit GEMM over its tap subset, writing every other pixel
  (``os = 2``); classes with no taps are zero-filled;
* dgrad can take the residual branch's gradient as an epilogue addend
  (``D = A.B^T + E``) — used where a tensor feeds both a conv and a skip path;
* wgrad: ``csrc/kernels/wgrad.hip`` — split-K MFMA GEMM over output pixels
  with ``ds_read_b64_tr_b16`` transposed operand reads; the partial sums are
  reduced straight into the weight's flat gradient view (direct-gradient
  protocol), so no dW tensor and no AccumulateGrad add exist.

The weight lives as ``[Cout, Cin, kh, kw]`` in channels_last memory, i.e.
physically ``[Cout][kh][kw][Cin]`` — exactly the K-contiguous B operand.
The 3-channel stride-2 stem runs as a stride-1 4x4 conv over its space-to-depth
input on the same kernels (``csrc/kernels/stem.hip``, ``_StemConvFn``).
"""
from __future__ import annotations

import math
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ..parallel.flat import direct_grad_view, notify_grad_ready

P, I = _lib.P, _lib.I
_lib.register("kfa_conv_igemm", [P, P, P, P] + [I] * 20 + [P, P, P, P, I, P, P, P, P])
_lib.register("kfa_conv_igemm_bnpro", [P] * 5 + [I] * 12 + [P, P])
_lib.register("kfa_zero_bf16", [P, _lib.L, P])
_lib.register("kfa_weight_transpose", [P, P] + [I] * 10 + [P])
_lib.register("kfa_weight_transpose_multi", [P, P, I, I, P])
_lib.register("kfa_wgrad_part_floats", [I] * 7, _lib.L)
_lib.register("kfa_conv_wgrad", [P, P, P, I, I, P] + [I] * 11 + [P])
_lib.register("kfa_bn_stats_partial", [P, P, _lib.L, I, P])
_lib.register("kfa_stem_s2d", [P, P, I, I, I, I, I, P])
_lib.register("kfa_stem_weight_s2d", [P, P, I, I, I, I, P])
_lib.register("kfa_stem_wgrad_fold", [P, P, I, I, I, I, I, I, P])

# Runtime switches (tests compare against the vendor path); env KFA_CONV_IGEMM=0 / KFA_WGRAD=0 disable.
ENABLED = os.environ.get("KFA_CONV_IGEMM", "1") != "0"
WGRAD_ENABLED = os.environ.get("KFA_WGRAD", "1") != "0"
# KFA_CONV_WGRAD_SIDE=1: conv weight gradients on the side stream (ops/streams.py),
# concurrent with the data-gradient chain (dgrad convs, BatchNorm backward passes)
WGRAD_SIDE = os.environ.get("KFA_CONV_WGRAD_SIDE", "0") == "1"


def igemm_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 and w.shape[2] == w.shape[3])


# 256x256 8-wave tiles for wide layers: opt-in (KFA_CONV_BIG=1).  On the ResNet-50 shapes they
# lose to the 4-wave 128x128 tiles (tools/bench_conv.py: fwd 4.76 -> 6.20 ms, dgrad 5.40 ->
# 7.09 ms per step): the late stages have too few 256x256 tiles to fill 256 CUs and convs
# have no split-K.  KFA_CONV_BIG_MINK: minimum reduction length K = R*S*C.
BIG = os.environ.get("KFA_CONV_BIG", "0") == "1"
BIG_MIN_K = int(os.environ.get("KFA_CONV_BIG_MINK", "256"))


# Forward tuner (like cudnn.benchmark, per layer shape): the implicit GEMM with the
# BatchNorm statistics fused in its epilogue vs the vendor (MIOpen) forward plus
# the separate statistics pass the BN then runs.  Measured once per shape on first
# use, outside any graph capture; env KFA_CONV_TUNE=0 keeps every layer on the
# implicit GEMM.  tools/bench_conv.py shows where MIOpen's forward wins: the
# compute-heavy 3x3 / K >= 1024 layers of the late stages (e.g. 256->256 3x3 at
# 14x14: 0.075 vs 0.110 ms), never the memory-bound expand 1x1s.
# Residual gradient of identity blocks formed in conv1's dgrad epilogue from the raw
# gradient + ReLU bits (GradJoin.deposit_masked); KFA_MASKED_RESIDUAL=0 writes it instead.
MASKED_RESIDUAL = os.environ.get("KFA_MASKED_RESIDUAL", "1") != "0"
TUNE = os.environ.get("KFA_CONV_TUNE", "0") == "1"  # opt-in: the own kernels win every ResNet-50 shape (10,003 vs 10,099 img/s with the vendor race on)
TUNE_LOG = os.environ.get("KFA_CONV_TUNE_LOG", "0") == "1"
_fwd_plan: dict = {}  # shape key -> True: vendor forward + BN stats pass


def _time_ms(fn, reps: int = 5) -> float:
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


_LOCKSTEP = False  # set by a data-parallel Engine: every rank of the default group runs the same step


def set_lockstep(on: bool) -> None:
    global _LOCKSTEP
    _LOCKSTEP = bool(on)


def _agree(hit: bool, device) -> bool:
    """Data-parallel ranks must run the same kernels: rank 0's tuning decision wins
    (every rank reaches each layer's first use in the same order, so this
    one-element broadcast is matched).  Only in lockstep jobs (``set_lockstep``,
    the collective Engine): async-PS workers share their default group with PS
    tasks that never run the model, so a broadcast there would never complete —
    each async worker keeps its own decision."""
    import torch.distributed as dist
    if not _LOCKSTEP or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return hit
    from ..parallel.comm import control_device  # the CPU unless the default group is torch's RCCL
    t = torch.tensor([1 if hit else 0], dtype=torch.int32, device=control_device(device))
    dist.broadcast(t, 0)
    return bool(t.item())


def _use_vendor_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, stats) -> bool:
    if not (TUNE and x.is_cuda):
        return False
    key = (tuple(x.shape), tuple(w.shape), stride, pad, stats is not None)
    hit = _fwd_plan.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return False
    with torch.no_grad():
        x, w = _cl(x), _cl(w)
        scratch = torch.zeros(_lib.lib().kfa_bn_slot_floats(w.shape[0]), dtype=torch.float32, device=x.device) \
            if stats is not None else None
        t_ours = _time_ms(lambda: conv_fwd(x, w, stride, pad, scratch))
        y = F.conv2d(x, w, None, stride, pad)
        t_vendor = _time_ms(lambda: F.conv2d(x, w, None, stride, pad))
        if stats is not None:
            M, C = y.numel() // y.shape[1], y.shape[1]
            t_vendor += _time_ms(lambda: _lib.call("kfa_bn_stats_partial", _lib.ptr(y), _lib.ptr(scratch), M, C,
                                                   _lib.stream()))
    hit = _fwd_plan[key] = _agree(t_vendor < 0.95 * t_ours, x.device)
    if TUNE_LOG:
        print(f"[kfa conv tune] x{tuple(x.shape)} w{tuple(w.shape)} s{stride} stats={stats is not None}: "
              f"igemm {t_ours:.3f} ms, vendor{'+stats' if stats is not None else ''} {t_vendor:.3f} ms -> "
              f"{'vendor' if hit else 'igemm'}", file=sys.stderr, flush=True)
    return hit


NARROW = int(os.environ.get("KFA_CONV_NARROW", "1"))  # tile variant for N <= 64: 1 = 128x64, 3 = 256x64
# ... for N <= 64 with a long reduction (K >= 512: the 3x3 64-channel convs, fwd and dgrad)
NARROW_LONGK = int(os.environ.get("KFA_CONV_NARROW_LONGK", str(NARROW)))


# 256x256 tiles where they win per shape (tools/bench_conv_tiles.py, bs 256): the
# memory-bound short reductions over many pixels (K <= 128, M >= 200704: the 56x56
# 64->256 expand forward, the 256->64 / 256->128 data gradients) — one block per CU
# streaming a 256-wide output tile keeps more of the epilogue's stores in flight
# (0.176 -> 0.163 ms, 0.283 -> 0.236 ms); every compute-bound shape loses there.
BIG_AUTO = os.environ.get("KFA_CONV_BIG_AUTO", "1") != "0"
BIG_AUTO_E = os.environ.get("KFA_CONV_BIG_AUTO_E", "1") != "0"  # also for launches with an addend


# Ping-pong 256x256 implicit GEMM (conv_pp_kernel, variant 4): "1" = every launch with
# N >= PP_MIN_N, "0" = never, "auto" = per launch shape from the committed routing table
# (ops/routes.py; timed at first use when the shape is not in it) vs the default tile.
# Per ResNet-50 shape (profiles/r5_conv_pp_layers.md): 1.4x on the 14x14 3x3s and the
# wide 1x1s, slower where 256x256 tiles leave CUs idle (7x7, N = 128).  "512": force the
# 512x128 ping-pong tile (variant 6, the 128-channel layers) instead.
PP = os.environ.get("KFA_CONV_PP", "auto")
PP_MIN_N = int(os.environ.get("KFA_CONV_PP_MIN_N", "256"))
_IG_VARIANT, _IG_STATS = 23, 24  # argument positions in kfa_conv_igemm
_pp_scratch: dict = {}


def _igemm(args: list, stats_t=None, kind: str = "conv") -> None:
    """One ``kfa_conv_igemm`` launch; with ``KFA_CONV_PP=auto`` the tile variant of this
    launch shape (geometry + epilogue features) is the routed one: the default tile vs
    the ping-pong kernel, from the table or timed once (statistics into a scratch
    slot buffer, so the real BatchNorm slots only see the real launch)."""
    N, K, C = args[16], args[10] * args[11] * args[7], args[7]
    narrow = N <= 64 and args[_IG_VARIANT] in (1, 3)
    # routed: every launch with whole 64-channel k-slices; the narrow tiles also for the
    # multi-tap slices of the space-to-depth stem (C = 16), where only they apply
    if PP == "auto" and N >= 64 and K > 0 and (C % 64 == 0 or narrow):
        from . import routes
        flags = tuple(int(args[i] is not None) for i in (3, _IG_STATS, 25, 31))
        key = tuple(args[4:23]) + flags
        dev = stats_t.device if stats_t is not None else torch.device("cuda", torch.cuda.current_device())
        sc = None
        if stats_t is not None:
            sc = _pp_scratch.get((stats_t.numel(), dev))
            if sc is None:
                sc = _pp_scratch[(stats_t.numel(), dev)] = torch.zeros_like(stats_t)

        def run(v):
            a = list(args)
            a[_IG_VARIANT] = v
            if sc is not None:
                a[_IG_STATS] = _lib.ptr(sc)
            return lambda: _lib.call("kfa_conv_igemm", *a)
        # every ping-pong form competes, even with part of its tile width empty: on the
        # 64-channel 3x3s the 512x128 tile (half empty) still beats the 128x64 one by 10 %
        # (profiles/r5_conv_pp_layers.md)
        cands = [("igemm", run(args[_IG_VARIANT]), args[_IG_VARIANT])]
        if C % 64 == 0:
            cands.append(("pp", run(4), 4))
            if N <= 512:  # 512 x 128 ping-pong: the 64 / 128-channel layers and narrow N <= 512 grids
                cands.append(("pp512", run(6), 6))
        if args[_IG_VARIANT] == 2:  # the static rule chose the 8-wave 256x256 tile: the 128x128 one competes too
            cands.append(("igemm128", run(0), 0))
        if narrow:  # narrow layers: the 128x64 and 256x64 tiles compete
            other = 3 if args[_IG_VARIANT] == 1 else 1
            cands.append(("igemm256x64" if other == 3 else "igemm128x64", run(other), other))
        i = routes.decide(kind, key, dev, [(n, f) for n, f, _ in cands])
        if i:
            args = list(args)
            args[_IG_VARIANT] = cands[i][2]
    _lib.call("kfa_conv_igemm", *args)


def _variant(M: int, N: int, K: int = 0, addend: bool = False) -> int:
    """Tile shape of one implicit-GEMM launch: M output pixels x N channels, reduction K."""
    if PP in ("1", "512") and N >= PP_MIN_N and K > 0:
        return 4 if PP == "1" else 6
    if N <= 64:
        return NARROW_LONGK if K >= 512 else NARROW
    if BIG and N % 256 == 0 and K >= BIG_MIN_K:
        return 2
    if BIG_AUTO and (BIG_AUTO_E or not addend) and N % 256 == 0 and 0 < K <= 128 and M >= 200704:
        return 2
    return 0


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, stats=None) -> torch.Tensor:
    """Forward conv; with ``stats`` (the BatchNorm slot workspace of Cout) the
    epilogue also accumulates the per-channel sum / sum of squares of the output
    for the BatchNorm that consumes it (``kfa_bn_fwd_train_prestats``)."""
    x, w = _cl(x), _cl(w)
    Nb, C, H, W = x.shape
    Co, _, R, S = w.shape
    Po = (H + 2 * pad - R) // stride + 1
    Qo = (W + 2 * pad - S) // stride + 1
    y = torch.empty((Nb, Co, Po, Qo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    _igemm([_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, Nb, H, W, C, Po, Qo, R, S, stride, 1,
            -pad, -pad, Co, Po, Qo, 1, 0, 0, Co, _variant(Nb * Po * Qo, Co, R * S * C), _lib.ptr(stats), None, None,
            None, 0, None, None, None, _lib.stream()], stats, "conv_fwd")
    return y


def bnpro_ok(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> bool:
    """``conv_fwd_bnpro`` covers this conv (and can write the normalised input as
    a side output): NHWC bf16, C % 64 == 0, stride 1, 'same' padding."""
    Co, C, R, S = w.shape
    return (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and C % 64 == 0 and C <= 2048
            and Co % 8 == 0 and stride == 1 and R == S and 2 * pad == R - 1)


def conv_fwd_bnpro(x: torch.Tensor, ss: torch.Tensor, w: torch.Tensor, stride: int, pad: int, stats=None,
                   y_out: "torch.Tensor | None" = None) -> torch.Tensor:
    """Forward conv of ``relu(x * scale + shift)`` (per channel; ``ss`` = [scale | shift],
    the BatchNorm's finalize output) with the BatchNorm-apply folded into the
    implicit GEMM's A-operand load (``kfa_conv_igemm_bnpro``).  ``y_out`` (same
    shape as ``x``) receives the normalised activation for the weight gradient."""
    x, w = _cl(x), _cl(w)
    Nb, C, H, W = x.shape
    Co, _, R, S = w.shape
    Po = (H + 2 * pad - R) // stride + 1
    Qo = (W + 2 * pad - S) // stride + 1
    y = torch.empty((Nb, Co, Po, Qo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    if y_out is not None and not y_out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_fwd_bnpro: y_out must be channels-last")
    _lib.call("kfa_conv_igemm_bnpro", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(ss), _lib.ptr(y_out), Nb, H, W,
              C, Po, Qo, R, S, stride, pad, Co, _variant(Nb * Po * Qo, Co, R * S * C), _lib.ptr(stats), _lib.stream())
    return y


def _transposed_weight(w: torch.Tensor, r0: int, dr: int, Rs: int, s0: int, ds: int, Ss: int) -> torch.Tensor:
    if Rs * Ss and getattr(w, "_kfa_flat", False) and BATCHED_TRANSPOSE:
        return _tcache.get(w, r0, dr, Rs, s0, ds, Ss)
    Co, Ci, R, S = w.shape
    wt = torch.empty((Ci, Rs, Ss, Co), dtype=w.dtype, device=w.device)
    if Rs * Ss:
        _lib.call("kfa_weight_transpose", _lib.ptr(w), _lib.ptr(wt), Co, R, S, Ci, r0, dr, Rs, s0, ds, Ss,
                  _lib.stream())
    return wt


BATCHED_TRANSPOSE = os.environ.get("KFA_BATCHED_TRANSPOSE", "1") != "0"


class _TransposeCache:
    """The dgrad operand ``W -> [Cin][taps][Cout]`` of every flat-buffer conv weight,
    refreshed by ONE batched launch at the first dgrad of each backward pass
    (the forward marks it stale; the weights are final by then).  A transpose
    met for the first time is computed on its own and joins the batch from the
    next step on."""

    def __init__(self):
        self.entries = {}      # key -> (w, wt, args)
        self.stale = True
        self._table = None     # (descs uint8 device tensor, first int32 device tensor, n, total)

    def mark_stale(self) -> None:
        self.stale = True

    def _build_table(self, device) -> None:
        import struct
        tdesc = _lib.lib().kfa_tdesc_bytes()
        blob, first, total = bytearray(), [], 0
        for w, wt, (Co, R, S, Ci, r0, dr, Rs, s0, ds, Ss) in self.entries.values():
            gx, gy = -(-Ci // 64), -(-Co // 64)  # weight_transpose_multi's 64 x 64 tiles
            rec = struct.pack("<QQ12i", w.data_ptr(), wt.data_ptr(), Co, R, S, Ci, r0, dr, Rs, s0, ds, Ss, gx, gy)
            blob += rec + bytes(tdesc - len(rec))
            first.append(total)
            total += gx * gy * Rs * Ss
        descs = torch.frombuffer(blob, dtype=torch.uint8).to(device)
        firsts = torch.tensor(first, dtype=torch.int32).to(device)
        self._table = (descs, firsts, len(first), total)

    def refresh(self, device) -> None:
        self.stale = False
        if not self.entries:
            return
        if self._table is None:
            self._build_table(device)
        descs, firsts, n, total = self._table
        _lib.call("kfa_weight_transpose_multi", _lib.ptr(descs), _lib.ptr(firsts), n, total, _lib.stream())

    def get(self, w, r0, dr, Rs, s0, ds, Ss) -> torch.Tensor:
        if self.stale:
            self.refresh(w.device)
        key = (w.data_ptr(), tuple(w.shape), r0, dr, Rs, s0, ds, Ss)
        hit = self.entries.get(key)
        if hit is not None:
            return hit[1]
        Co, Ci, R, S = w.shape
        wt = torch.empty((Ci, Rs, Ss, Co), dtype=w.dtype, device=w.device)
        _lib.call("kfa_weight_transpose", _lib.ptr(w), _lib.ptr(wt), Co, R, S, Ci, r0, dr, Rs, s0, ds, Ss,
                  _lib.stream())
        self.entries[key] = (w, wt, (Co, R, S, Ci, r0, dr, Rs, s0, ds, Ss))
        self._table = None
        return wt


_tcache = _TransposeCache()


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride: int, pad: int, addend=None,
               bn=None, addend_mask=None) -> torch.Tensor:
    """``bn``: a ``batchnorm.BnBwdLink`` of the BatchNorm whose output is this conv's
    input — the epilogue then also accumulates that BN's backward statistics.
    ``addend_mask``: uint8 ReLU bits (one per element of ``addend``, channels-last
    order, LSB first); the epilogue adds ``addend * mask`` instead of ``addend``."""
    dy, w = _cl(dy), _cl(w)
    Nb, Co, Po, Qo = dy.shape
    _, Ci, R, S = w.shape
    H, W = x_shape[2], x_shape[3]
    dx = torch.empty((Nb, Ci, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
    E = None if addend is None else _cl(addend)
    EM = None if E is None else addend_mask
    if EM is not None and (EM.dtype != torch.uint8 or EM.numel() * 8 != dx.numel()):
        raise ValueError(f"conv_dgrad: addend mask of {EM.numel()} bytes for {dx.numel()} elements")
    st = _lib.stream()
    bn_args = (None, None, None, None, 0, None, None)
    bn_ws = None
    if bn is not None:
        from .batchnorm import bn_slot_workspace
        bn_ws = bn_slot_workspace(Ci, dy.device)
        bn_args = (_lib.ptr(bn_ws), _lib.ptr(bn.x), _lib.ptr(bn.y), _lib.ptr(bn.mean),
                   int(bn.relu), _lib.ptr(bn.ss), _lib.ptr(bn.mb))
        bn.prestats = True
    if stride == 1:
        wt = _transposed_weight(w, 0, 1, R, 0, 1, S)
        _igemm([_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), _lib.ptr(E), Nb, Po, Qo, Co, H, W, R, S,
                1, -1, pad, pad, Ci, H, W, 1, 0, 0, Ci, _variant(Nb * H * W, Ci, R * S * Co, E is not None), *bn_args,
                _lib.ptr(EM), st], bn_ws, "conv_dgrad")
        return dx
    # stride s: output parity classes.  For class (ph, pw) the rows h = s*i + ph
    # receive taps r with (ph + pad - r) % s == 0, from dY row i + (ph + pad - r)/s.
    for ph in range(stride):
        r0 = (ph + pad) % stride
        Rs = len(range(r0, R, stride))
        Hc = len(range(ph, H, stride))
        for pw in range(stride):
            s0 = (pw + pad) % stride
            Ss = len(range(s0, S, stride))
            Wc = len(range(pw, W, stride))
            if Hc == 0 or Wc == 0:
                continue
            # a class no tap reaches (1x1/s2: 3 of 4) runs with K = 0: the kernel
            # writes zeros (or the addend) through the same strided output mapping
            wt = _transposed_weight(w, r0, stride, Rs, s0, stride, Ss) if Rs * Ss else w
            oa_h = (ph + pad - r0) // stride
            oa_w = (pw + pad - s0) // stride
            _igemm([_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), _lib.ptr(E), Nb, Po, Qo, Co, Hc, Wc,
                    Rs, Ss, 1, -1, oa_h, oa_w, Ci, H, W, stride, ph, pw, Ci,
                    _variant(Nb * Hc * Wc, Ci, Rs * Ss * Co, E is not None),
                    *bn_args, _lib.ptr(EM), st], bn_ws, "conv_dgrad")
    return dx


def conv_wgrad_vendor(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    _, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1],
                                                   False, [0, 0], 1, [False, True, False])
    return gw


def wgrad_ok(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor) -> bool:
    return (WGRAD_ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16
            and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0
            and dy.shape[0] * dy.shape[2] * dy.shape[3] < (1 << 24))


def wgrad_into(x, dy, out, Nb, H, W, Ci, P_, Q_, Co, R, S, stride, pad, accumulate: bool) -> None:
    """out (+)= dW  for NHWC x [Nb,H,W,Ci] / dy [Nb,P,Q,Co]; out is [Co][R][S][Ci] (bf16 or fp32)."""
    nfl = _lib.lib().kfa_wgrad_part_floats(Nb, P_, Q_, Co, R, S, Ci)
    # one split-K partial workspace per stream (BERT's encoder wgrads run on the side stream, ops/streams.py)
    part = _lib.workspace(nfl * 4, x.device, f"wgrad_part{_lib.stream() or 0}").view(torch.float32)
    _lib.call("kfa_conv_wgrad", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(out), int(out.dtype == torch.float32),
              int(accumulate), _lib.ptr(part), Nb, H, W, Ci, P_, Q_, Co, R, S, stride, pad, _lib.stream())


_wgrad_plan: dict = {}  # shape key -> True: vendor weight gradient


def _use_vendor_wgrad(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> bool:
    """Weight-gradient side of the per-shape tuner: split-K MFMA wgrad vs the vendor's
    (plus the add into the fp32 flat gradient it then needs).  On ResNet-50 the vendor
    wins the 64-channel 3x3 at 56x56 (0.17 vs 0.23 ms)."""
    if not (TUNE and x.is_cuda):
        return False
    key = (tuple(x.shape), tuple(w.shape), stride, pad)
    hit = _wgrad_plan.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return False
    Nb, Ci, H, W = x.shape
    Co, _, R, S = w.shape
    with torch.no_grad():
        acc = torch.zeros(w.shape, dtype=torch.float32, device=x.device).contiguous(memory_format=torch.channels_last)
        t_ours = _time_ms(lambda: wgrad_into(x, dy, acc, Nb, H, W, Ci, dy.shape[2], dy.shape[3], Co, R, S, stride, pad,
                                             True))
        t_vendor = _time_ms(lambda: acc.add_(conv_wgrad_vendor(x, dy, w, stride, pad)))
    hit = _wgrad_plan[key] = _agree(t_vendor < 0.95 * t_ours, x.device)
    if TUNE_LOG:
        print(f"[kfa conv tune] wgrad x{tuple(x.shape)} w{tuple(w.shape)} s{stride}: ours {t_ours:.3f} ms, "
              f"vendor {t_vendor:.3f} ms -> {'vendor' if hit else 'ours'}", file=sys.stderr, flush=True)
    return hit


def conv_wgrad(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor, stride: int, pad: int, wparam=None):
    """Weight gradient.  Returns None when it was accumulated directly into the
    parameter's flat gradient buffer (and the bucket notified), else dW."""
    if not wgrad_ok(x, dy, w):
        return conv_wgrad_vendor(x, dy, w, stride, pad)
    x, dy = _cl(x), _cl(dy)
    Nb, Ci, H, W = x.shape
    Co, _, R, S = w.shape
    P_, Q_ = dy.shape[2], dy.shape[3]
    target = direct_grad_view(wparam) if wparam is not None else None
    direct = target is not None and target.dtype in (torch.bfloat16, torch.float32) and \
        target.is_contiguous(memory_format=torch.channels_last)
    if _use_vendor_wgrad(x, dy, w, stride, pad):
        gw = conv_wgrad_vendor(x, dy, w, stride, pad)
        if not direct:
            return gw
        target.add_(gw)
        notify_grad_ready(wparam)
        return None
    if direct:
        wgrad_into(x, dy, target, Nb, H, W, Ci, P_, Q_, Co, R, S, stride, pad, accumulate=True)
        notify_grad_ready(wparam)
        return None
    dw = torch.empty_like(w, memory_format=torch.channels_last)
    wgrad_into(x, dy, dw, Nb, H, W, Ci, P_, Q_, Co, R, S, stride, pad, accumulate=False)
    return dw


class GradJoin:
    """Fuses the gradient SUM of a tensor that feeds two branches into a conv's dgrad.

    ``xb = join.branch(x)`` is an alias of ``x`` whose gradient is *deposited*
    here instead of flowing back to ``x``; the conv built with
    ``conv2d(x, w, ..., join=join)`` then computes ``dx = dgrad(dy) + deposit``
    in its epilogue (``E`` operand of ``kfa_conv_igemm``), so autograd never runs
    the separate add kernel.  Autograd's ready-queue order (latest-created node
    first) runs the branch's backward before the conv's; if it ever does not,
    the branch simply returns its gradient to autograd (correct, just unfused).

    A join lives for ONE forward/backward: models create a fresh one per forward
    (``models/resnet.py``), so no deposit can leak into the next step.  Its
    backward runs once: ``retain_graph=True`` re-runs and partial
    ``torch.autograd.grad`` calls over the block are not supported (a second
    pass would find the state already consumed).
    """

    __slots__ = ("grad", "mask", "state", "fused")

    def __init__(self):
        self.grad = None
        self.mask = None  # with grad: ReLU bits; the residual gradient is grad * mask (see deposit)
        self.state = "empty"  # empty -> deposited -> empty | consumer-first
        self.fused = False    # set by the consuming conv's forward (HIP path only)

    def branch(self, x):
        if not (torch.is_grad_enabled() and x.requires_grad and self.fused):
            return x
        return _Branch.apply(x, self)

    def deposit_masked(self, grad, mask) -> bool:
        """Called by the backward of a BN + residual + ReLU whose residual input is
        this branch: hand over the raw output gradient and the ReLU bits instead of
        materialising grad * mask (the consuming dgrad epilogue applies the mask).
        False when the consumer already ran (the caller returns a real gradient)."""
        if self.state != "empty" or not self.fused or not MASKED_RESIDUAL:
            return False
        self.grad, self.mask, self.state = grad, mask, "deposited"
        return True


class _Branch(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, join):
        ctx.join = join
        ctx.set_materialize_grads(False)  # None = the gradient was deposited (GradJoin.deposit_masked)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        j = ctx.join
        if g is None:
            return None, None
        if j.state == "consumer-first":
            j.state = "empty"
            return g, None
        j.grad, j.state = g, "deposited"
        return None, None


# KFA_CONV_BNPRO=0: lazy BatchNorm outputs are always materialised by the apply pass
BNPRO = os.environ.get("KFA_CONV_BNPRO", "1") != "0"
_bnpro_choice = {}


def _use_bnpro(lz, x, w, stride, pad, stats) -> bool:
    """Fold the lazy BatchNorm's apply into this conv (``conv_fwd_bnpro``)?  Per shape, the
    faster of (apply pass + conv) and the fused conv, timed once at first use (scratch
    outputs and statistics; rank 0's choice everywhere).  Measured: a win for the 1x1
    bn2 -> conv3 layers up to 256 channels, a loss for every 3x3 (the transform is redone
    per tap) — ``profiles/r4_bn_apply_prologue.md``."""
    if not (BNPRO and bnpro_ok(x, w, stride, pad) and not torch.cuda.is_current_stream_capturing()):
        return False
    key = (tuple(x.shape), tuple(w.shape), stride, pad, stats is not None)
    hit = _bnpro_choice.get(key)
    if hit is None:
        M, C = x.numel() // x.shape[1], x.shape[1]
        yy = torch.empty_like(lz.x)
        st = None
        if stats is not None:
            st = torch.zeros_like(stats)
        Co = w.shape[0]

        def sep():
            _lib.call("kfa_bn_apply_ss", _lib.ptr(lz.x), _lib.ptr(yy), _lib.ptr(lz.ss), M, C, 1, _lib.stream())
            conv_fwd(yy, w, stride, pad, st)

        from . import routes  # committed table first, else timed (median of 3 x 30 launches)
        i = routes.decide("bnpro", key, x.device,
                          [("sep", sep), ("pro", lambda: conv_fwd_bnpro(lz.x, lz.ss, w, stride, pad, st, yy))],
                          margin=0.98)
        hit = _bnpro_choice[key] = i == 1
        del yy, st, Co
    return hit


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, join, stats, vendor=False, lazy=None):
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad, ctx.join = stride, pad, join
        ctx.wparam = w  # the Parameter itself (for the direct flat-gradient write)
        ctx.bn_link = getattr(x, "_kfa_bn_link", None)  # x = output of a BatchNorm (see conv_dgrad)
        if ctx.bn_link is not None:
            ctx.bn_link.convs += 1
        _tcache.mark_stale()  # weights may have changed since the last backward
        if lazy is not None:  # x is a lazy BN output: this launch also writes it (for the wgrad)
            lazy.pending = False
            return conv_fwd_bnpro(lazy.x, lazy.ss, w, stride, pad, stats, x)
        if vendor:
            return _cl(F.conv2d(_cl(x), _cl(w), None, stride, pad))
        return conv_fwd(x, w, stride, pad, stats)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            addend = addend_mask = None
            bn_link = ctx.bn_link if (ctx.bn_link is not None and ctx.bn_link.convs == 1) else None
            j = ctx.join
            if j is not None:
                if j.state == "deposited":
                    addend, addend_mask, j.grad, j.mask, j.state = j.grad, j.mask, None, None, "empty"
                else:
                    j.state = "consumer-first"
                    # this epilogue sees only part of x's gradient: the BN whose output x
                    # is must compute its backward statistics itself
                    bn_link = None
            if w.shape[0] % 64 == 0 and w.shape[1] % 8 == 0:
                dx = conv_dgrad(dy, w, x.shape, ctx.stride, ctx.pad, addend, bn_link, addend_mask)
            else:
                dx = torch.nn.grad.conv2d_input(x.shape, w, dy, ctx.stride, ctx.pad)
                if addend is not None and addend_mask is not None:
                    addend = apply_bit_mask(addend, addend_mask)
                if addend is not None:
                    dx = dx + addend
        if ctx.needs_input_grad[1]:
            if WGRAD_SIDE and x.is_cuda:
                from . import streams as _streams
                dw = _streams.run_on_side(lambda: conv_wgrad(x, dy, w, ctx.stride, ctx.pad, ctx.wparam), x.device,
                                          (x, dy, w))
                if dw is not None:  # a returned gradient is consumed on the main stream
                    torch.cuda.current_stream(x.device).wait_stream(_streams.side_stream(x.device))
            else:
                dw = conv_wgrad(x, dy, w, ctx.stride, ctx.pad, ctx.wparam)
        return dx, dw, None, None, None, None, None, None


def apply_bit_mask(t: torch.Tensor, bits: torch.Tensor) -> torch.Tensor:
    """``t * mask`` for a ReLU bit mask over ``t``'s channels-last elements (LSB first)."""
    t = _cl(t)
    shifts = torch.arange(8, device=bits.device, dtype=torch.uint8)
    m = ((bits.view(-1, 1) >> shifts) & 1).view(-1)
    flat = t.permute(0, 2, 3, 1).reshape(-1) if t.dim() == 4 else t.reshape(-1)
    out = torch.where(m.bool(), flat, torch.zeros((), dtype=t.dtype, device=t.device))
    if t.dim() == 4:
        n, c, h, w_ = t.shape
        return out.view(n, h, w_, c).permute(0, 3, 1, 2)
    return out.view_as(t)


def stem_ok(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> bool:
    """A few-channel stride-2 conv (the 7x7 ResNet stem) the space-to-depth path covers."""
    return (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.shape[1] <= 4 and stride == 2 and w.shape[2] == w.shape[3] and w.shape[2] <= 8
            and (x.shape[2] + 2 * pad) % 2 == 0 and (x.shape[3] + 2 * pad) % 2 == 0 and w.shape[0] % 64 == 0)


def stem_inputs(x: torch.Tensor, w: torch.Tensor, pad: int):
    """Space-to-depth views of the stem (``csrc/kernels/stem.hip``): xs [N,16,Hs,Ws], ws [Co,16,Rs,Ss]."""
    x, w = _cl(x), _cl(w)
    Nb, C, H, W = x.shape
    Co, _, R, S = w.shape
    Hs, Ws = (H + 2 * pad) // 2, (W + 2 * pad) // 2
    Rs, Ss = (R + 1) // 2, (S + 1) // 2
    xs = torch.empty((Nb, 16, Hs, Ws), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    ws = torch.empty((Co, 16, Rs, Ss), dtype=w.dtype, device=w.device, memory_format=torch.channels_last)
    st = _lib.stream()
    _lib.call("kfa_stem_s2d", _lib.ptr(x), _lib.ptr(xs), Nb, H, W, C, pad, st)
    _lib.call("kfa_stem_weight_s2d", _lib.ptr(w), _lib.ptr(ws), Co, R, S, C, st)
    return xs, ws


class _StemConvFn(torch.autograd.Function):
    """The 3-channel stride-2 stem as a stride-1 4x4 conv over the space-to-depth
    input: forward and weight gradient on the same MFMA kernels as every other
    conv (no vendor kernel, BatchNorm statistics fused)."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, stats):
        xs, ws = stem_inputs(x, w, pad)
        y = conv_fwd(xs, ws, 1, 0, stats)
        ctx.save_for_backward(xs, w)
        ctx.x_shape, ctx.stride, ctx.pad = x.shape, stride, pad
        ctx.wparam = w
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, w = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.nn.grad.conv2d_input(ctx.x_shape, w, dy, ctx.stride, ctx.pad)
        if ctx.needs_input_grad[1]:
            dy = _cl(dy)
            Nb, _, Hs, Ws = xs.shape
            Co, C, R, S = w.shape
            Rs, Ss = (R + 1) // 2, (S + 1) // 2
            dws = torch.empty((Co, Rs, Ss, 16), dtype=torch.float32, device=dy.device)
            wgrad_into(xs, dy, dws, Nb, Hs, Ws, 16, dy.shape[2], dy.shape[3], Co, Rs, Ss, 1, 0, accumulate=False)
            target = direct_grad_view(ctx.wparam)
            direct = target is not None and target.dtype in (torch.bfloat16, torch.float32) and \
                target.is_contiguous(memory_format=torch.channels_last)
            out = target if direct else torch.empty_like(w, memory_format=torch.channels_last)
            _lib.call("kfa_stem_wgrad_fold", _lib.ptr(dws), _lib.ptr(out), int(out.dtype == torch.float32),
                      int(direct), Co, R, S, C, _lib.stream())
            if direct:
                notify_grad_ready(ctx.wparam)
            else:
                dw = out
        return dx, dw, None, None, None


def conv2d(x, w, stride: int = 1, pad: int = 0, join: "GradJoin | None" = None, bn_stats=False):
    """``bn_stats``: the caller guarantees a training-mode ``BatchNorm2dAct``
    consumes the output next; the epilogue then accumulates its statistics and
    the output is tagged ``_kfa_prestats`` (the BN skips its stats pass).  A
    string names the slot workspace (``ops.batchnorm.bn_slot_workspace`` tag)
    for a BN whose finalize runs later than the next BN's (the downsample BN of
    ``bn_act_dual``); True = the shared one."""
    tag = bn_stats if isinstance(bn_stats, str) else "bn_slots"
    lz = getattr(x, "_kfa_lazy", None)
    if lz is not None and lz.pending and join is None and igemm_ok(x, w):
        stats = None
        if bn_stats:
            from .batchnorm import bn_slot_workspace
            stats = bn_slot_workspace(w.shape[0], x.device, tag)
        if _use_bnpro(lz, x, w, stride, pad, stats):
            y = _ConvFn.apply(x, w, stride, pad, None, stats, False, lz)
            if stats is not None:
                y._kfa_prestats = True
                y._kfa_prestats_tag = tag
            return y
    if lz is not None and lz.pending:
        from .batchnorm import materialize
        materialize(x)
    if stem_ok(x, w, stride, pad) and join is None:
        stats = None
        if bn_stats:
            from .batchnorm import bn_slot_workspace
            stats = bn_slot_workspace(w.shape[0], x.device, tag)
        y = _StemConvFn.apply(x, w, stride, pad, stats)
        if stats is not None:
            y._kfa_prestats = True
            y._kfa_prestats_tag = tag
        return y
    if igemm_ok(x, w):
        if join is not None:
            join.fused = True
        stats = None
        if bn_stats:
            from .batchnorm import bn_slot_workspace
            stats = bn_slot_workspace(w.shape[0], x.device, tag)
        vendor = _use_vendor_fwd(x, w, stride, pad, stats)
        if vendor:
            stats = None  # the BN runs its own statistics pass
        y = _ConvFn.apply(x, w, stride, pad, join, stats, vendor)
        if stats is not None:
            y._kfa_prestats = True
            y._kfa_prestats_tag = tag
        return y
    return F.conv2d(x, w, None, stride, pad)  # unfused: join.branch() is a no-op alias


class Conv2d(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 bias: bool = False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.stride = stride
        self.padding = padding
        w = torch.empty(out_channels, in_channels, kernel_size, kernel_size)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = nn.Parameter(w.contiguous(memory_format=torch.channels_last))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None

    def forward(self, x, join: "GradJoin | None" = None, bn_stats=False):
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        y = conv2d(x, w, self.stride, self.padding, join, bn_stats if self.bias is None else False)
        if self.bias is not None:
            y = y + self.bias.to(y.dtype).view(1, -1, 1, 1)
        return y

    def extra_repr(self) -> str:
        return (f"{self.in_channels}, {self.out_channels}, k={self.kernel_size}, s={self.stride}, "
                f"p={self.padding}, bias={self.bias is not None}")
