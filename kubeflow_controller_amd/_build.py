"""In-tree build of the native parts.

* ``_native_runtime`` — C++ control-plane runtime (core in
  ``csrc/runtime/runtime_core.h``, bindings in ``runtime.cpp``), compiled with
  g++ against pybind11.
* ``parallel/_kfc_comm.so`` — the first-party collective layer (``csrc/comm/comm.cpp``:
  bootstrap, RCCL resolved at run time, host-TCP backend for CPU tests), g++.
* ``ops/_hip_kernels.so`` — the hand-written CDNA4 kernels (``csrc/kernels/*.hip``)
  compiled by ``hipcc --offload-arch=gfx950`` into ONE shared object with a C
  ABI; Python binds it with ``ctypes`` (``ops/_lib.py``), so no torch headers
  are compiled and rebuilds take seconds.
* ``build/sanitize/{runtime,comm}_selftest_{asan,tsan}`` — the runtime core's native
  self-test (``csrc/runtime/selftest.cpp``) and the collective layer's
  (``csrc/comm/comm_selftest.cpp``: 3 host-backend ranks as threads) under
  ASan+UBSan and TSan (``--sanitize``; host code only).

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
    srcs = [src, os.path.join(CSRC, "runtime", "runtime_core.h")]
    tgt = runtime_target()
    with _lock:
        if not force and _up_to_date(tgt, srcs):
            return tgt
        cxx = os.environ.get("CXX", "g++")
        tmp = tgt + f".tmp{os.getpid()}"
        cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-function",
               f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
               src, "-o", tmp, "-lpthread"]
        _run(cmd, quiet=True)
        os.replace(tmp, tgt)
        _write_stamp(tgt, srcs)
    return tgt


def comm_target() -> str:
    return os.path.join(PKG, "parallel", "_kfc_comm.so")


def build_comm(force: bool = False) -> str:
    """The first-party collective layer (``csrc/comm/comm.cpp``: TCP bootstrap,
    RCCL backend resolved at run time, host-TCP backend for CPU) as a C-ABI
    shared object bound with ctypes (``parallel/comm.py``).  Plain g++: it
    includes no HIP / RCCL header (RCCL is dlopen'ed), so it builds and its host
    backend runs on a machine without ROCm devices."""
    src = os.path.join(CSRC, "comm", "comm.cpp")
    tgt = comm_target()
    with _lock:
        if not force and _up_to_date(tgt, [src]):
            return tgt
        cxx = os.environ.get("CXX", "g++")
        tmp = tgt + f".tmp{os.getpid()}"
        _run([cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
              "-fvisibility=hidden", src, "-o", tmp, "-ldl", "-lpthread"], quiet=True)
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


SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}


def sanitize_cxx() -> str:
    """ROCm's clang++ when present: gcc-11's TSan does not intercept
    ``pthread_cond_clockwait`` (what ``condition_variable::wait_for`` uses), so
    it reports a false "double lock" on every timed wait; clang's runtime does."""
    for c in (os.environ.get("KFA_SANITIZE_CXX"), "/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++")):
        if c and os.path.exists(c):
            return c
    return os.environ.get("CXX", "g++")


SELFTESTS = {
    "runtime": [os.path.join(CSRC, "runtime", "selftest.cpp"), os.path.join(CSRC, "runtime", "runtime_core.h")],
    "comm": [os.path.join(CSRC, "comm", "comm_selftest.cpp"), os.path.join(CSRC, "comm", "comm.cpp")],
}


def sanitize_target(kind: str, canary: bool = False, target: str = "runtime") -> str:
    return os.path.join(ROOT, "build", "sanitize", f"{target}_selftest_{kind}" + ("_canary" if canary else ""))


def build_sanitized(kind: str, force: bool = False, canary: bool = False, target: str = "runtime") -> str:
    """Compile a native self-test under one sanitizer (host code only):
    ``target`` = ``runtime`` (work queue, limiters, expectations, launcher) or
    ``comm`` (the collective layer's host backend, 3 ranks as threads).

    ``canary=True`` also compiles in a deliberate defect (a data race under
    TSan, a heap overflow under ASan) so a test can prove the tool is live."""
    srcs = SELFTESTS[target]
    tgt = sanitize_target(kind, canary, target)
    with _lock:
        if not force and _up_to_date(tgt, srcs):
            return tgt
        os.makedirs(os.path.dirname(tgt), exist_ok=True)
        tmp = tgt + f".tmp{os.getpid()}"
        cmd = [sanitize_cxx(), "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Wall",
               "-Wno-unused-function", *SANITIZERS[kind], *(["-DKFA_SELFTEST_INJECT"] if canary else []),
               srcs[0], "-o", tmp, "-lpthread", *(["-ldl"] if target == "comm" else [])]
        _run(cmd, quiet=True)
        os.replace(tmp, tgt)
        _write_stamp(tgt, srcs)
    return tgt


def run_sanitized(kind: str, timeout: float = 300.0, canary: bool = False,
                  target: str = "runtime") -> subprocess.CompletedProcess:
    """Build and run one sanitizer self-test; a sanitizer report makes it exit
    23 (ASan / UBSan build) or 25 (TSan build)."""
    exe = build_sanitized(kind, canary=canary, target=target)
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)  # a preloaded runtime ahead of libasan/libtsan aborts the run
    if kind == "asan":  # UBSan shares the common flags (exitcode) of the ASan runtime
        env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:halt_on_error=1:exitcode=23"
        env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    else:
        env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=25:second_deadlock_stack=1"
    return subprocess.run([exe], capture_output=True, text=True, timeout=timeout, env=env)


def build_all(force: bool = False) -> None:
    build_runtime(force)
    build_comm(force)
    build_kernels(force)


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        rc = 0
        for target, kind in [(t, k) for t in SELFTESTS for k in SANITIZERS]:
            r = run_sanitized(kind, target=target)
            sys.stdout.write(f"[{target} {kind}] " + r.stdout)
            if r.returncode != 0:
                sys.stderr.write(r.stderr[-8000:])
                rc = r.returncode
        sys.exit(rc)
    build_all(force="--force" in sys.argv)
    print("built:", runtime_target(), kernels_target())
