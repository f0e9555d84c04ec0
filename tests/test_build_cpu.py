"""Build-level checks that run without a GPU (the driver's CPU round): the HIP
kernel library links every kernel's host launch stub, and the launchers the
Python ops bind are exported."""
import os
import shutil
import subprocess

import pytest

from kubeflow_controller_amd import _build


def _kernels_so():
    path = _build.kernels_target()
    if not os.path.exists(path):
        pytest.skip("HIP kernel library not built (run __graft_entry__.build())")
    return path


def test_no_undefined_kernel_launch_stubs():
    """clang's host pass silently drops the stub of a templated kernel it cannot
    instantiate; such a library only fails at dlopen on the GPU box."""
    so = _kernels_so()
    if not shutil.which("nm"):
        pytest.skip("nm not available")
    out = subprocess.run(["nm", "-u", so], capture_output=True, text=True).stdout
    assert "__device_stub__" not in out, [l for l in out.splitlines() if "__device_stub__" in l]


def test_bound_launchers_are_exported():
    """Every kfa_* symbol the Python ops register must be defined in the library."""
    so = _kernels_so()
    if not shutil.which("nm"):
        pytest.skip("nm not available")
    from kubeflow_controller_amd.ops import _lib
    import kubeflow_controller_amd.ops.batchnorm  # noqa: F401  (each module registers its launchers)
    import kubeflow_controller_amd.ops.conv  # noqa: F401
    import kubeflow_controller_amd.ops.gemm  # noqa: F401
    import kubeflow_controller_amd.ops.loss  # noqa: F401
    import kubeflow_controller_amd.ops.optim  # noqa: F401
    import kubeflow_controller_amd.ops.pool  # noqa: F401
    import kubeflow_controller_amd.ops.transformer  # noqa: F401
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    defined = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = sorted(n for n in _lib._SIGS if n not in defined)
    assert not missing, missing
