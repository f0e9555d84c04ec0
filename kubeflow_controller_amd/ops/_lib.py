"""ctypes binding of ``ops/_hip_kernels.so`` (all ``csrc/kernels/*.hip``).

Every launcher has a C ABI ``int kfa_<op>(..., hipStream_t)`` returning the HIP
status of its launches (0 = ok).  Tensors are passed as raw device pointers and
the CURRENT torch stream is passed explicitly, so the kernels compose with
torch's stream semantics and hipGraph capture.

There is no silent fallback: on a GPU process, a missing or unloadable kernel
library raises.  (CPU-only processes never touch this module.)
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import _build

_lib = None
_lock = threading.Lock()

P = ctypes.c_void_p
L = ctypes.c_long
I = ctypes.c_int
F = ctypes.c_float

# name -> argtypes (restype is int status unless listed in _RESTYPE)
_SIGS = {
    "kfa_bn_slot_floats": [I],
    "kfa_bn_coef_floats": [I],
    "kfa_bn_fwd_train": [P, P, P, P, P, P, P, P, P, P, P, L, I, F, F, I, P, P],
    "kfa_bn_fwd_eval": [P, P, P, P, P, P, P, P, L, I, F, I, P],
    "kfa_bn_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, L, I, I, I, P, P, P],
}
_RESTYPE = {"kfa_bn_slot_floats": L, "kfa_bn_coef_floats": L}


def register(name: str, argtypes, restype=I) -> None:
    """Kernel modules declare their C signatures here at import time."""
    _SIGS[name] = argtypes
    if restype is not I:
        _RESTYPE[name] = restype
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.argtypes = argtypes
        fn.restype = restype


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.kernels_target()
        if os.environ.get("KFA_KERNELS_SO"):  # A/B experiments: another in-tree build of the same sources
            path = os.path.join(os.path.dirname(path), os.environ["KFA_KERNELS_SO"])
        elif not os.path.exists(path) or os.environ.get("KFA_REBUILD_KERNELS") == "1":
            _build.build_kernels()
        h = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, I)
        _lib = h
    return _lib


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP kernel {what} failed with status {rc}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


_ws = {}


def workspace(nbytes: int, device, tag: str = "default") -> torch.Tensor:
    """Grow-only per-(device, tag) scratch buffer (never freed mid-step)."""
    key = (str(device), tag)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        # zero-initialised: BN's slot accumulators rely on it (kernels re-zero after use)
        buf = torch.zeros(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf
