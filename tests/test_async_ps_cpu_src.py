"""With device signalling (KFA_PS_DEVICE_SIGNAL=1) the device-resident async PS's
steady-state push / pull path has no host synchronisation: the
hand-offs are interprocess HIP events (parallel/async_ps.py module doc) and the
only host waits live in ``_host_wait``, which runs only on the host-waited
protocol (the measured-faster default) / invisible-GPU fallback.  Both protocols
run on the GPU in tests/test_async_ps_gpu.py."""
import inspect
import re

from kubeflow_controller_amd.parallel import async_ps as A

HOST_SYNC = re.compile(r"\.synchronize\(|torch\.cuda\.synchronize|\.item\(\)|\.cpu\(\)|\.tolist\(\)")


def _src(fn):
    return inspect.getsource(fn)


def test_steady_state_methods_have_no_host_sync():
    for fn in (A.DeviceAsyncPSClient.push, A.DeviceAsyncPSClient.pull, A.DeviceAsyncPSServer._apply,
               A.DeviceAsyncPSServer._acc_add, A.DeviceAsyncPSServer._recv_grad):
        bad = [l.strip() for l in _src(fn).splitlines() if HOST_SYNC.search(l)]
        assert not bad, (fn.__qualname__, bad)


def test_host_waits_only_on_the_fallback_branches():
    after = _src(A.DeviceAsyncPSServer._after_update)
    assert "if self.signal:" in after and "_host_wait(" in after.split("else:", 1)[1]
    push = _src(A.DeviceAsyncPSClient.push)
    # the host wait covers only devices collected for PUSH_DEV (not self.sig[k])
    assert "not self.sig[k]" in push and "_host_wait(" in push
    assert "PUSH_SIG if self.sig[k] else PUSH_DEV" in push
    assert ".synchronize()" in _src(A._host_wait)


def test_signal_switch(monkeypatch):
    """Opt-in: measured slower than the host-waited protocol (module doc)."""
    monkeypatch.delenv("KFA_PS_DEVICE_SIGNAL", raising=False)
    assert not A.device_signal_enabled()
    monkeypatch.setenv("KFA_PS_DEVICE_SIGNAL", "1")
    assert A.device_signal_enabled()
