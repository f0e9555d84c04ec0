"""Every ctypes signature the Python ops register matches the C ABI of the HIP
kernel library (``KFA_API`` declarations in ``csrc/kernels/*.hip``): parameter
count and the width / kind of each one.  A short argtypes list is not an error
to ctypes — the extra arguments are passed as C ints, so a 64-bit stream handle
or pointer past the list is silently truncated."""
import ctypes
import glob
import importlib
import os
import pkgutil
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_signatures():
    sigs = {}
    pat = re.compile(r"KFA_API\s+([\w\s\*]+?)\s*\b(kfa_\w+)\s*\(([^)]*)\)", re.S)
    for f in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")):
        src = open(f).read()
        for ret, name, params in pat.findall(src):
            params = " ".join(params.split())
            sigs[name] = [p.strip() for p in params.split(",")] if params.strip() not in ("", "void") else []
    return sigs


def _kind(decl: str):
    t = decl.rsplit(" ", 1)[0] if " " in decl else decl
    if "*" in decl or "hipStream_t" in decl:
        return ctypes.c_void_p
    if "unsigned long long" in t or "uint64_t" in t:
        return ctypes.c_ulonglong
    if re.search(r"\blong\b", t):
        return ctypes.c_long
    if re.search(r"\bfloat\b", t):
        return ctypes.c_float
    if re.search(r"\bdouble\b", t):
        return ctypes.c_double
    return ctypes.c_int


def test_registered_ctypes_signatures_match_the_c_abi():
    import kubeflow_controller_amd.ops as ops_pkg
    from kubeflow_controller_amd.ops import _lib
    for m in pkgutil.iter_modules(ops_pkg.__path__):
        if m.name.startswith("_hip"):  # the kernel library itself (ctypes, not a Python module)
            continue
        importlib.import_module(f"kubeflow_controller_amd.ops.{m.name}")
    importlib.import_module("kubeflow_controller_amd.parallel.embedding")  # registers its sparse kernels too
    csigs = _c_signatures()
    assert len(csigs) > 40, "KFA_API declarations not found"
    bad = []
    for name, argtypes in _lib._SIGS.items():
        assert name in csigs, f"{name} is registered but has no KFA_API declaration"
        want = [_kind(p) for p in csigs[name]]
        got = list(argtypes)
        if len(got) != len(want):
            bad.append(f"{name}: {len(got)} argtypes for {len(want)} C parameters")
            continue
        for i, (g, w) in enumerate(zip(got, want)):
            same = g is w or (g in (ctypes.c_long, ctypes.c_longlong) and w is ctypes.c_long) \
                or (g is ctypes.c_ulonglong and w is ctypes.c_ulonglong) or (g is ctypes.c_uint and w is ctypes.c_int)
            if not same:
                bad.append(f"{name} arg {i} ({csigs[name][i]}): registered {g.__name__}, C wants {w.__name__}")
    assert not bad, "\n".join(bad)
