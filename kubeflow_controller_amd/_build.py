"""In-tree build of the native parts.

* ``_native_runtime`` — C++ control-plane runtime (``csrc/runtime/runtime.cpp``),
  compiled with g++ against pybind11.
* ``ops/_hip_kernels.so`` — the hand-written CDNA4 kernels (``csrc/kernels/*.hip``)
  compiled by ``hipcc --offload-arch=gfx950`` into ONE shared object with a C
  ABI; Python binds it with ``ctypes`` (``ops/_lib.py``), so no torch headers
  are compiled and rebuilds take seconds.
* ``parallel/_comm.so`` — C++ bucket planner / flat-buffer packing helpers
  (``csrc/comm/*.cpp``).

Everything lands inside the package directory so it travels with the repo
snapshot to the GPU box (``gpurun``) and is visible as an in-tree ``.so``.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
import threading

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
_lock = threading.Lock()


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _stamp(paths) -> str:
    h = hashlib.sha1()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()[:16]


def _up_to_date(target: str, sources) -> bool:
    stamp = target + ".stamp"
    if not os.path.exists(target) or not os.path.exists(stamp):
        return False
    with open(stamp) as f:
        return f.read().strip() == _stamp(sources)


def _write_stamp(target: str, sources) -> None:
    with open(target + ".stamp", "w") as f:
        f.write(_stamp(sources))


def _run(cmd, quiet=False):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if not quiet and r.stderr.strip():
        sys.stderr.write(r.stderr)


def runtime_target() -> str:
    return os.path.join(PKG, "_native_runtime" + _ext_suffix())


def build_runtime(force: bool = False) -> str:
    import pybind11
    src = os.path.join(CSRC, "runtime", "runtime.cpp")
    tgt = runtime_target()
    with _lock:
        if not force and _up_to_date(tgt, [src]):
            return tgt
        cxx = os.environ.get("CXX", "g++")
        tmp = tgt + f".tmp{os.getpid()}"
        cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function",
               f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
               src, "-o", tmp, "-lpthread"]
        _run(cmd, quiet=True)
        os.replace(tmp, tgt)
        _write_stamp(tgt, [src])
    return tgt


def kernels_target() -> str:
    return os.path.join(PKG, "ops", "_hip_kernels.so")


def kernel_sources():
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) +
                  glob.glob(os.path.join(CSRC, "kernels", "*.h")))


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _check_stubs(so: str) -> None:
    """Fail the build if a kernel's host launch stub is missing from the .so
    (clang's host pass silently drops the stub of a templated kernel whose body
    it cannot instantiate; the library then only fails at dlopen on the GPU box)."""
    nm = shutil.which("nm")
    if not nm:
        return
    out = subprocess.run([nm, "-u", so], capture_output=True, text=True).stdout
    bad = [l.split()[-1] for l in out.splitlines() if "__device_stub__" in l]
    if bad:
        raise RuntimeError(f"HIP kernel build: undefined launch stubs in {so}: {bad}")


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    """Compile every ``csrc/kernels/*.hip`` for gfx950 and link one .so."""
    srcs = kernel_sources()
    hips = [s for s in srcs if s.endswith(".hip")]
    tgt = kernels_target()
    with _lock:
        if not force and _up_to_date(tgt, srcs):
            return tgt
        objdir = os.path.join(ROOT, "build", "kernels")
        os.makedirs(objdir, exist_ok=True)
        cc = hipcc()
        flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                 "-Wno-unused-result", f"-I{os.path.join(CSRC, 'kernels')}"]
        procs = []
        objs = []
        for s in hips:
            o = os.path.join(objdir, os.path.basename(s) + ".o")
            objs.append(o)
            procs.append((s, subprocess.Popen([cc, *flags, "-c", s, "-o", o],
                                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
            if len([p for p in procs if p[1].poll() is None]) >= jobs:
                procs[0][1].wait()
        errs = []
        for s, p in procs:
            out, err = p.communicate()
            if p.returncode != 0:
                errs.append(f"--- {s}\n{out}\n{err}")
        if errs:
            raise RuntimeError("HIP kernel build failed:\n" + "\n".join(errs))
        tmp = tgt + f".tmp{os.getpid()}"
        _run([cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp], quiet=True)
        _check_stubs(tmp)
        os.replace(tmp, tgt)
        _write_stamp(tgt, srcs)
    return tgt


def comm_target() -> str:
    return os.path.join(PKG, "parallel", "_comm" + _ext_suffix())


def build_comm(force: bool = False) -> str:
    import pybind11
    srcs = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    if not srcs:
        return ""
    tgt = comm_target()
    with _lock:
        if not force and _up_to_date(tgt, srcs):
            return tgt
        tmp = tgt + f".tmp{os.getpid()}"
        cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC",
               f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", *srcs, "-o", tmp]
        _run(cmd, quiet=True)
        os.replace(tmp, tgt)
        _write_stamp(tgt, srcs)
    return tgt


def build_all(force: bool = False) -> None:
    build_runtime(force)
    build_comm(force)
    build_kernels(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", runtime_target(), comm_target(), kernels_target())
