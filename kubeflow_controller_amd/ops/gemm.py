"""Dense GEMM + fused epilogues on the hand-written MFMA kernel
(``csrc/kernels/gemm.hip``) — SURVEY §2.6 K1 "GEMM + bias (+ReLU/GELU) epilogue".

``gemm_nt(a, b)`` computes ``epilogue(a @ b.T)`` for bf16 ``a [M, K]`` and
``b [N, K]`` (both K-contiguous): the forward of a dense layer (``b`` = the
weight as stored, ``[out, in]``) and its dgrad (``b`` = :func:`transpose` of
the weight).  Epilogue options, all fused into the tile write-out:

* ``bias`` (fp32, added to the fp32 accumulator before any rounding);
* ``addend`` (bf16 ``[M, N]``, e.g. a residual-gradient join);
* ``want_z`` (also return the pre-activation, for the backward);
* ``act`` (``gelu`` / ``tanh`` / ``relu``);
* ``zin`` + ``dact`` (multiply by ``act'(zin)``: the backward of the NEXT
  layer's activation, fused into this dgrad);
* ``dbias`` (fp32 ``[N]``: column sums of the output accumulated into a
  bias-gradient vector, e.g. a flat-buffer gradient view).

``gemm_reference`` is the plain PyTorch fp32 definition the tests compare to.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib
from . import conv as _conv  # noqa: F401  (registers kfa_weight_transpose)

P, I = _lib.P, _lib.I
_lib.register("kfa_gemm_nt", [P] * 9 + [I] * 10 + [P])
_lib.register("kfa_gemm_dpart_floats", [I, I, I, I], restype=_lib.L)
_lib.register("kfa_gemm_pick_bn", [I, I])
_lib.register("kfa_gemm_ppp", [P, P, P] + [I] * 9 + [P, _lib.L, I, P])
_lib.register("kfa_gemm_ppp_ws_bytes", [I] * 5, restype=_lib.L)
_lib.register("kfa_gemm_ppp_pick_bn", [I, I])
_lib.register("kfa_gemm_skinny", [P, P, P, P] + [I] * 7 + [P, _lib.L, P])
_lib.register("kfa_gemm_ppp_gelu", [P] * 5 + [I] * 6 + [P])
_lib.register("kfa_gemm_ppp_relu", [P] * 4 + [I] * 6 + [P])
_lib.register("kfa_gemm_ppw_relu", [P] * 4 + [I] * 7 + [P])
_lib.register("kfa_gemm_ppw_dact", [P] * 7 + [I] * 8 + [P])
_lib.register("kfa_gemm_ppw_dact_part_floats", [I, I], _lib.L)
_lib.register("kfa_gemm_skinny_ws_bytes", [I] * 4, restype=_lib.L)

ACTS = {None: 0, "none": 0, "gelu": 1, "tanh": 2, "relu": 3}
# Which dense-layer GEMMs run on this kernel (KFA_GEMM):
#   "auto"   (default) every shape picks own-vs-library per shape, timed once at
#            first use (an own kernel must beat hipBLASLt by 1 %);
#   "own"    every shape an own kernel covers runs on the fastest OWN kernel
#            (persistent / wave-specialised / skinny GEMMs); hipBLASLt is timed for
#            the tuner log only.  Same box, 2 rounds: BERT-base 8,879-9,003 vs
#            9,223-9,228 seq/s with "auto" (the FFN forward GEMMs lose 10-15 % to
#            hipBLASLt); W&D 27.66 vs 27.71 M ex/s;
#   "1"      every projection (forward and dgrad), encoder layers included;
#   "fused"  only the ones whose epilogue replaces a separate pass: the FFN-up
#            forward (bias + GELU + pre-activation) and its dgrad (GELU' +
#            bias-gradient column sums);
#   "0"      none (hipBLASLt via torch.mm / addmm for all of them).
# Measured on MI355X (tools/bench_gemm.py, tools/gpu_bert_gemm.sh; docs/kernels.md).
_ROUTE = os.environ.get("KFA_GEMM", "auto")
ROUTE_LAYERS = _ROUTE == "1"
ROUTE_FUSED = _ROUTE in ("1", "fused")
ROUTE_AUTO = _ROUTE in ("auto", "own")
OWN_ONLY = _ROUTE == "own"
TUNE_LOG = os.environ.get("KFA_GEMM_TUNE_LOG", "0") == "1"
_choice: dict = {}


def prefer_own(kind: str, key: tuple, device, run_own, run_lib) -> bool:
    """Per-shape own-kernel vs library choice (``KFA_GEMM=auto``): both forms timed
    once at first use, outside any graph capture, and rank 0's decision applied on
    every rank (data-parallel ranks must run the same kernels).  ``run_own`` /
    ``run_lib`` must be free of side effects (they run a few times)."""
    k = (kind,) + tuple(key)
    hit = _choice.get(k)
    if hit is not None:
        return hit
    from . import routes  # committed per-arch table first, else timed (median of 3 x 30 launches)
    i = routes.decide(kind, key, device, [("library", run_lib), ("own", run_own)], margin=0.97, log=TUNE_LOG)
    if torch.cuda.is_current_stream_capturing() and i == 0:
        return False  # not cached: decided for real outside the capture
    hit = _choice[k] = i == 1
    return hit


def gemm_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Operands the kernel takes: bf16 CUDA matrices, K-contiguous, K / N / row
    strides multiples of 8 (16-B LDS-DMA pieces), 16-B aligned, every operand
    within 32-bit buffer offsets."""
    return (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1] and a.shape[1] % 8 == 0
            and b.shape[0] % 8 == 0 and a.shape[0] > 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0
            and b.data_ptr() % 16 == 0 and a.shape[0] * b.shape[0] * 2 < (1 << 31)
            and a.shape[0] * a.stride(0) * 2 < (1 << 31) and b.shape[0] * b.stride(0) * 2 < (1 << 31))


def _check_mn(t, M, N, what):
    if t is not None and (t.dtype != torch.bfloat16 or tuple(t.shape) != (M, N) or not t.is_contiguous()
                          or t.data_ptr() % 16):
        raise ValueError(f"gemm_nt: {what} must be a contiguous bf16 [{M}, {N}] tensor")


def _check_vec(t, N, what):
    if t is not None and (t.dtype != torch.float32 or t.numel() != N or not t.is_contiguous()
                          or t.data_ptr() % 16):
        raise ValueError(f"gemm_nt: {what} must be a contiguous, 16-B aligned fp32 [{N}] vector")


# Kernel variant: 0 = one 8-wave block per 256 x bn tile (128 KB ring: one block
# per CU), 1 = persistent blocks carrying the LDS ring across tiles, 3 = 256 x 128
# blocks on a 3-slot ring (72 KB: two blocks per CU, so one block's barriers and
# epilogue run under the other's MFMAs — the pick for short k-loops), 4 = as 3 with
# four 128 x 64 waves.  KFA_GEMM_VARIANT overrides; tools/bench_gemm.py compares.
# 5 / 6 = 256 x 256 ping-pong (two wave groups one barrier apart; 6 with
# non-temporal C stores), K % 64 == 0: the fastest main loop (1.1-1.4 PFLOP/s
# without its epilogue), but its C write is not overlapped with MFMA work, so
# it wins only where the k-loop is long or the output wide (K >= 2048 or
# N >= 3072; tools/bench_gemm.py, docs/kernels.md).  None = pick per shape.
_VAR_ENV = os.environ.get("KFA_GEMM_VARIANT")
PERSISTENT = int(_VAR_ENV) if _VAR_ENV else None


def pick_variant(M: int, N: int, K: int) -> int:
    if K % 64 == 0 and (K >= 2048 or N >= 3072):
        return 6
    return 3


def gemm_nt(a, b, *, bias=None, act=None, addend=None, want_z=False, zin=None, dact=None, dbias=None, out=None,
            bn: int = 0, persistent=None):
    """``(C, Z)`` with ``C = epilogue(a @ b.T)`` (see module doc); ``Z`` is None unless ``want_z``."""
    if not gemm_ok(a, b):
        raise ValueError(f"gemm_nt: unsupported operands {tuple(a.shape)}/{a.dtype} x {tuple(b.shape)}/{b.dtype}")
    M, K = a.shape
    N = b.shape[0]
    c = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _check_mn(c, M, N, "out")
    _check_mn(addend, M, N, "addend")
    _check_mn(zin, M, N, "zin")
    _check_vec(bias, N, "bias")
    if dbias is not None and (dbias.dtype != torch.float32 or dbias.numel() != N or not dbias.is_contiguous()):
        raise ValueError(f"gemm_nt: dbias must be a contiguous fp32 [{N}] vector")
    if (zin is None) != (dact in (None, "none")):
        raise ValueError("gemm_nt: zin and dact go together")
    z = torch.empty_like(c) if want_z else None
    variant = persistent if persistent is not None else PERSISTENT
    variant = pick_variant(M, N, K) if variant is None else int(variant)
    dpart = None
    if dbias is not None:  # partial column sums + one reduce (no per-column atomics)
        nf = _lib.lib().kfa_gemm_dpart_floats(M, N, int(bn), variant)
        dpart = _lib.workspace(4 * nf, a.device, "gemm_dbias") if nf else None
    _lib.call("kfa_gemm_nt", _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), _lib.ptr(addend), _lib.ptr(bias), _lib.ptr(z),
              _lib.ptr(zin), _lib.ptr(dbias), _lib.ptr(dpart), M, N, K, a.stride(0), b.stride(0), N, ACTS[act],
              ACTS[dact], int(bn), variant, _lib.stream())
    return c, z


def gemm_ppp(a, b, *, out=None, blocks: int = 0, probe: int = 0, bn: int = 0, split: bool = True):
    """``a @ b.T`` (bf16) on the persistent ping-pong kernel (``csrc/kernels/gemm_ppp.hip``):
    one block per CU sweeps its tiles as one continuous k-tile pipeline, each tile's
    C written from the accumulators during the next tile's first k-tile.  K % 8 == 0, K >= 128
    (a partial last 64-deep k-tile reads zeros past K).
    ``blocks`` > 0 caps the persistent grid (tests: many tiles per block).  ``probe=1``:
    timing probe with every C store dropped (C is left unwritten).  ``probe`` 9 / 10:
    the wave-specialised 256 x 256 kernel (plain / non-temporal C stores); 11 / 12:
    its 256 x 192 three-phase form (``gemm_ppw3_kernel``).  ``bn``: tile
    width 256 or 192 (0 = the kernel's pick: 192-wide tiles where N % 192 == 0 and
    256-wide ones would leave a partial last round, e.g. N = 768 at M = 32768).
    ``split``: the tiles past the grid's last full round are cut into k-ranges
    run by several blocks (fp32 partials combined in-kernel), so every CU runs
    about the same number of k-tiles — e.g. 384 tiles on 256 CUs: one full tile
    plus half a tile each instead of two tiles on half the CUs."""
    if not gemm_ok(a, b) or a.shape[1] < 128:
        raise ValueError(f"gemm_ppp: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    c = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _check_mn(c, M, N, "out")
    nb = _lib.lib().kfa_gemm_ppp_ws_bytes(M, N, K, int(bn), int(blocks)) if split else 0
    ws = _lib.workspace(nb, a.device, f"ppp_ws{_lib.stream() or 0}") if nb > 0 else None
    _lib.call("kfa_gemm_ppp", _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), M, N, K, a.stride(0), b.stride(0), N,
              int(blocks), int(probe), int(bn), _lib.ptr(ws), nb, int(not split), _lib.stream())
    return c


def ppw_dact_ok(a, b, zin) -> bool:
    """Operands :func:`gemm_ppw_dact` takes."""
    return (ppp_ok(a, b) and zin is not None and zin.dtype == torch.bfloat16 and zin.is_contiguous()
            and tuple(zin.shape) == (a.shape[0], b.shape[0]) and zin.data_ptr() % 16 == 0)


def gemm_ppw_dact(a, b, zin, bias=None, dbias=None, *, nt: bool = False, accumulate: bool = True):
    """``dz = (a @ b.T) * gelu'(zin + bias)`` (bf16) from ONE launch of the
    wave-specialised persistent GEMM with the GELU-backward epilogue
    (``gemm_ppw_kernel<..., DACT>``): no separate activation-gradient pass.
    ``dbias`` (fp32 [N]) (+)= the column sums of dz (epilogue band partials + one
    small reduce launch, fixed order)."""
    if not ppw_dact_ok(a, b, zin):
        raise ValueError(f"gemm_ppw_dact: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    _check_vec(bias, N, "bias")
    c = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    part = None
    if dbias is not None:
        _check_vec(dbias, N, "dbias")
        part = _lib.workspace(_lib.lib().kfa_gemm_ppw_dact_part_floats(M, N) * 4, a.device,
                              f"ppw_dact{_lib.stream() or 0}")
    _lib.call("kfa_gemm_ppw_dact", _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), _lib.ptr(zin), _lib.ptr(bias),
              _lib.ptr(part), _lib.ptr(dbias), int(accumulate), M, N, K, a.stride(0), b.stride(0), N, int(nt),
              _lib.stream())
    return c


SKINNY_MAX_M = 16384  # the 256 x 64-tile kernel is a tuner candidate up to this many rows


def ppp_gelu_ok(a, b, bias) -> bool:
    """Operands :func:`gemm_ppp_gelu` takes."""
    return (ppp_ok(a, b) and b.shape[0] <= 8192 and bias is not None and bias.dtype == torch.float32
            and bias.is_contiguous() and bias.numel() == b.shape[0])


def gemm_ppp_gelu(a, b, bias):
    """``(y, z)`` with ``z = a @ b.T + bias`` (bf16: the pre-activation, bias included)
    and ``y = gelu(z)``, from ONE launch of the persistent GEMM with the bias + GELU
    epilogue (``gemm_ppp_kernel<..., GELU>``): no separate bias / activation pass."""
    if not ppp_gelu_ok(a, b, bias):
        raise ValueError(f"gemm_ppp_gelu: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    z = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    y = torch.empty_like(z)
    _lib.call("kfa_gemm_ppp_gelu", _lib.ptr(a), _lib.ptr(b), _lib.ptr(z), _lib.ptr(y), _lib.ptr(bias), M, N, K,
              a.stride(0), b.stride(0), N, _lib.stream())
    return y, z


def gemm_ppp_relu(a, b, bias):
    """``relu(a @ b.T + bias)`` (bf16) from ONE launch of the persistent GEMM with the
    bias + ReLU epilogue (``gemm_ppp_kernel<..., ACT = 2>``): no bias / activation pass
    and no pre-activation write — the backward takes the ReLU mask from the output."""
    if not ppp_gelu_ok(a, b, bias):
        raise ValueError(f"gemm_ppp_relu: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _lib.call("kfa_gemm_ppp_relu", _lib.ptr(a), _lib.ptr(b), _lib.ptr(y), _lib.ptr(bias), M, N, K,
              a.stride(0), b.stride(0), N, _lib.stream())
    return y


def gemm_ppw_relu(a, b, bias, nt: bool = False):
    """``relu(a @ b.T + bias)`` (bf16) from ONE launch of the wave-specialised persistent
    GEMM (``gemm_ppw_kernel<NT, false, 2>``): the store waves add the bias to the bf16
    product and clamp — the C stores stay off the DMA waves' counter, as in the plain
    ``ppw256`` variant (``nt``: non-temporal stores)."""
    if not ppp_gelu_ok(a, b, bias) or bias.data_ptr() % 16:
        raise ValueError(f"gemm_ppw_relu: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    y = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _lib.call("kfa_gemm_ppw_relu", _lib.ptr(a), _lib.ptr(b), _lib.ptr(y), _lib.ptr(bias), M, N, K,
              a.stride(0), b.stride(0), N, int(nt), _lib.stream())
    return y


def skinny_ok(a, b) -> bool:
    """Operands :func:`gemm_skinny` takes: N % 4 == 0 (bf16, K-contiguous); tuned for
    M <= SKINNY_MAX_M (one 256-row band for the ResNet FC, a few dozen for BERT's MLM head)."""
    return (a.is_cuda and b.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1] and 0 < a.shape[0] <= SKINNY_MAX_M
            and a.shape[1] % 8 == 0 and b.shape[0] % 4 == 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and b.shape[0] * b.stride(0) * 2 < (1 << 31))


def gemm_skinny(a, b, bias=None, *, splits: int = 0, out=None):
    """``a @ b.T (+ bias)`` (bf16 out, fp32 bias) on the split-K skinny kernel
    (``csrc/kernels/gemm_skinny.hip``): 256 x 64 output tiles over 256-row bands, the
    reduction cut into slices run by separate blocks when there are few tiles,
    partials summed in slice order by the last-arriving slice of each tile.
    ``splits`` 0 = about one block per CU."""
    if not skinny_ok(a, b):
        raise ValueError(f"gemm_skinny: unsupported operands {tuple(a.shape)} x {tuple(b.shape)}")
    M, K = a.shape
    N = b.shape[0]
    _check_vec(bias, N, "bias")
    c = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _check_mn(c, M, N, "out")
    nb = _lib.lib().kfa_gemm_skinny_ws_bytes(M, N, K, int(splits))
    ws = _lib.workspace(nb, a.device, f"skinny_ws{_lib.stream() or 0}") if nb > 0 else None
    _lib.call("kfa_gemm_skinny", _lib.ptr(a), _lib.ptr(b), _lib.ptr(c), _lib.ptr(bias), M, N, K, a.stride(0),
              b.stride(0), N, int(splits), _lib.ptr(ws), nb, _lib.stream())
    return c


def skinny_splits(a, b):
    """``(name, splits)`` forms of :func:`gemm_skinny` worth timing for ``a @ b.T``:
    the kernel's own pick (about one block per CU) and fixed 4 / 8 slices — fewer
    slices leave the last-arriving slice less partial data to sum."""
    M, K = a.shape
    N = b.shape[0]
    nks = K // 64
    tiles = -(-M // 256) * -(-N // 64)
    out = [("skinny", 0)]
    if tiles * 8 <= 256:  # fixed splits only where the tiles alone leave most CUs idle
        for s in (4, 8):
            if 2 * s <= nks:
                out.append((f"skinny-s{s}", s))
    return out


def ppp_ok(a, b) -> bool:
    """Operands :func:`gemm_ppp` takes (plain ``a @ b.T``, bf16 out)."""
    return gemm_ok(a, b) and a.shape[1] >= 128


def pick_fastest(kind: str, key: tuple, device, candidates) -> int:
    """Index of the fastest of ``candidates`` (``[(name, fn), ...]``, index 0 =
    the library form) for this shape: the committed routing table's pick
    (``ops/routes.py``), else timed once at first use outside any graph capture;
    rank 0's choice is applied on every rank.  An own kernel must beat the library
    by 1 % to be picked (timing noise never flips a tie to it)."""
    k = (kind,) + tuple(key)
    hit = _choice.get(k)
    if hit is not None:
        return hit
    from . import routes  # committed per-arch table first, else timed (median of 3 x 30 launches)
    i = routes.decide(kind, key, device, candidates, margin=1e9 if OWN_ONLY else 0.99, log=TUNE_LOG)
    if torch.cuda.is_current_stream_capturing() and i == 0:
        return 0
    _choice[k] = i
    return i


def _ppp_candidates(a, b):
    """Persistent-GEMM variants worth timing for ``a @ b.T``: 256-wide tiles with
    and without the split remainder, 192-wide tiles where N % 192 == 0."""
    M, K = a.shape
    N = b.shape[0]
    L = _lib.lib()
    c = [("ppp256", lambda: gemm_ppp(a, b, bn=256, split=False)),
         # wave-specialised stores: group 0 all LDS-DMA, group 1 all C stores (plain / non-temporal)
         ("ppw256", lambda: gemm_ppp(a, b, probe=9, split=False)),
         ("ppw256-nt", lambda: gemm_ppp(a, b, probe=10, split=False))]
    if L.kfa_gemm_ppp_ws_bytes(M, N, K, 256, 0) > 0:
        c.append(("ppp256-split", lambda: gemm_ppp(a, b, bn=256)))
    if N % 192 == 0:
        c.append(("ppp192", lambda: gemm_ppp(a, b, bn=192)))
        # wave-specialised 256 x 192 three-phase tiles (gemm_ppw3_kernel): N = 768 at
        # M = 32768 is 512 tiles = exactly two per CU
        c.append(("ppw192", lambda: gemm_ppp(a, b, probe=11, split=False)))
        c.append(("ppw192-nt", lambda: gemm_ppp(a, b, probe=12, split=False)))
    return c


def mm_auto(a, w, kind: str = "proj"):
    """``a @ w.T`` (bf16): the persistent MFMA GEMM variant that measured fastest
    for this shape when it beats hipBLASLt (timed once at first use, rank 0's
    choice applied everywhere — :func:`pick_fastest`), else the library.
    ``KFA_GEMM=0`` forces the library."""
    if ROUTE_AUTO and ppp_ok(a, w):
        cands = [("hipblaslt", lambda: torch.mm(a, w.t()))] + _ppp_candidates(a, w)
        if skinny_ok(a, w):
            cands += [(n, (lambda s: lambda: gemm_skinny(a, w, splits=s))(s)) for n, s in skinny_splits(a, w)]
        i = pick_fastest(kind, (a.shape[0], w.shape[0], a.shape[1]), a.device, cands)
        if i:
            return cands[i][1]()
    return torch.mm(a, w.t())


def dgrad_auto(dz, w, kind: str = "proj_dgrad"):
    """``dz @ w`` (the data gradient of ``y = x @ w.T``): the fastest own MFMA GEMM
    on the transposed weight (the persistent kernel's variants; the split-K skinny
    kernel for M <= 256) where it beats hipBLASLt for this shape, else the library.
    Flat-buffer weights take their transpose from the step's batched transpose
    cache (one launch per backward for every such weight, ``ops/conv.py``)."""
    M, K = dz.shape if dz.dim() == 2 else (0, 0)
    N = w.shape[1] if w.dim() == 2 else 0
    if (ROUTE_AUTO and dz.is_cuda and dz.dim() == 2 and w.dim() == 2 and dz.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and dz.is_contiguous() and dz.data_ptr() % 16 == 0 and K == w.shape[0]
            and K % 8 == 0 and N % 8 == 0 and M > 0
            and max(M * N, M * K, N * K) * 2 < (1 << 31)):
        k = (kind, M, N, K)
        if _choice.get(k) == 0:
            return torch.mm(dz, w)
        wt = transpose_cached(w)
        own = []
        if K >= 128:
            own += _ppp_candidates(dz, wt)
        if skinny_ok(dz, wt):
            own += [(n, (lambda s: lambda: gemm_skinny(dz, wt, splits=s))(s)) for n, s in skinny_splits(dz, wt)]
        if own:
            cands = [("hipblaslt", lambda: torch.mm(dz, w))] + own
            i = pick_fastest(kind, (M, N, K), dz.device, cands)
            if i:
                return own[i - 1][1]()
    return torch.mm(dz, w)


def transpose_cached(w: torch.Tensor) -> torch.Tensor:
    """``w.T`` contiguous: from the per-step batched transpose cache for a flat-buffer
    (optimizer-updated) weight, else a fresh :func:`transpose`."""
    if getattr(w, "_kfa_flat", False) and w.is_contiguous():
        from .conv import _tcache, BATCHED_TRANSPOSE
        if BATCHED_TRANSPOSE:
            R, C = w.shape
            return _tcache.get(w.view(R, C, 1, 1), 0, 1, 1, 0, 1, 1).view(C, R)
    return transpose(w)


def mark_weights_stale() -> None:
    """The weights may have changed since the last backward (a forward is running):
    the cached transposes are refreshed at the next backward's first dgrad."""
    from .conv import _tcache
    _tcache.mark_stale()


def transpose(w: torch.Tensor) -> torch.Tensor:
    """Contiguous ``w.T`` of a bf16 ``[R, C]`` matrix on the LDS-tiled HIP transpose
    (the dgrad B operand: ``dx = dy · W`` is ``gemm_nt(dy, transpose(W))``)."""
    R, C = w.shape
    w = w.contiguous()
    wt = torch.empty(C, R, dtype=w.dtype, device=w.device)
    _lib.call("kfa_weight_transpose", _lib.ptr(w), _lib.ptr(wt), R, 1, 1, C, 0, 1, 1, 0, 1, 1, _lib.stream())
    return wt


def _act(z, act):
    if act == "gelu":
        return F.gelu(z)
    if act == "tanh":
        return torch.tanh(z)
    if act == "relu":
        return torch.relu(z)
    return z


def _act_grad(z, act):
    zz = z.detach().float().requires_grad_()
    _act(zz, act).sum().backward()
    return zz.grad


def gemm_reference(a, b, bias=None, act=None, addend=None, zin=None, dact=None):
    """Plain PyTorch fp32 ``(C, Z)`` of :func:`gemm_nt`."""
    v = a.float() @ b.float().t()
    if bias is not None:
        v = v + bias.float()
    if addend is not None:
        v = v + addend.float()
    z = v
    v = _act(v, act)
    if zin is not None:
        v = v * _act_grad(zin, dact)
    return v, z
