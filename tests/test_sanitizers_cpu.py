"""Sanitizer builds of the native control-plane runtime.

The runtime core (``csrc/runtime/runtime_core.h``: work queue, rate limiters,
expectations, process launcher) is compiled WITHOUT Python into
``csrc/runtime/selftest.cpp`` under ASan+UBSan and under TSan, and the
self-test drives it concurrently (producers x workers over a small key space,
shutdown while blocked, queue churn, concurrent expectations, spawn/kill).
A canary build with a deliberate defect proves each sanitizer is live.

The collective layer (``csrc/comm/comm.cpp``: sockets, partial-I/O offsets, the
per-communicator mutex) gets the same treatment: ``csrc/comm/comm_selftest.cpp``
runs 3 host-backend ranks as threads of one process through every collective
with rank-distinct values (element-wise checks), hands each communicator to a
second thread mid-run, and exercises the size-mismatch / bootstrap-timeout
error paths — under ASan+UBSan and TSan.

The reference has no race detector at all (``Makefile:22-29``: plain
``go build``, no ``-race``).  Host code only — nothing here touches a GPU.
"""
import os
import shutil

import pytest

from kubeflow_controller_amd import _build

_cxx = _build.sanitize_cxx()
pytestmark = pytest.mark.skipif(not (os.path.exists(_cxx) or shutil.which(_cxx)), reason="no C++ compiler")


@pytest.mark.parametrize("target", ["runtime", "comm"])
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_selftest_clean_under_sanitizer(kind, target):
    r = _build.run_sanitized(kind, target=target)
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    assert "0 failed" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-6000:]


@pytest.mark.parametrize("kind,code,needle", [("tsan", 25, "data race"), ("asan", 23, "heap-buffer-overflow")])
def test_sanitizer_canary_is_caught(kind, code, needle):
    r = _build.run_sanitized(kind, canary=True)
    assert r.returncode == code, (r.returncode, r.stderr[-3000:])
    assert needle in r.stderr
