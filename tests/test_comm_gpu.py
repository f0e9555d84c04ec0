"""First-party communicator on the GPU: the RCCL backend of csrc/comm/comm.cpp at
world 1 (one MI355X per box: RCCL refuses two ranks on one device, the multi-rank
semantics are covered against gloo by tests/test_comm_cpu.py on its host backend).
Checks the TCP bootstrap + ncclCommInitRank path, every collective on device
buffers through the communicator's own stream, the event hand-off back to the
caller's stream, and that librccl and the comm library are what ran."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def comm():
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.comm import Communicator
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    c = Communicator.create(store, 0, 1, torch.device("cuda", torch.cuda.current_device()), advertise_host="127.0.0.1",
                            timeout_s=120)
    yield c
    c.destroy()


def test_rccl_backend_is_mapped(comm):
    from kubeflow_controller_amd.parallel import comm as C
    assert comm.backend == "rccl"
    maps = open("/proc/self/maps").read()
    assert "_kfc_comm.so" in maps and "librccl" in maps
    assert C.lib().kfc_rccl_version() > 0
    comm.check()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.int64])
def test_rccl_world1_collectives(comm, dt):
    d = comm.device
    x = (torch.randn(100003, device=d) * 50).to(dt)
    a = x.clone()
    comm.all_reduce(a)
    assert torch.equal(a, x)
    out = torch.empty_like(x)
    comm.reduce_scatter_tensor(out, x.clone())
    assert torch.equal(out, x)
    out = torch.empty_like(x)
    comm.all_gather_into_tensor(out, x)
    assert torch.equal(out, x)
    b = x.clone()
    comm.broadcast(b, 0)
    comm.reduce(b, 0)
    assert torch.equal(b, x)
    rows = x[:100000].reshape(1000, 100)
    o = torch.empty_like(rows)
    comm.all_to_all_single(o, rows, [1000], [1000])
    assert torch.equal(o, rows)
    comm.barrier()


def test_bringup_probe_passes_on_rccl(comm):
    """make_comm's bring-up probe (every collective the training paths use, on
    rank-distinct values) passes on the RCCL backend at world 1 — the probe itself
    (its dtypes, stream syncs, all-to-all splits) runs on the device path it guards."""
    from kubeflow_controller_amd.parallel.comm import _probe
    assert _probe(comm, comm.device, 1, 0, a2a=True) == ""


def test_rccl_async_event_handoff(comm):
    """async_op: the collective runs on the communicator's stream after the
    producer kernel; wait() orders the consumer after it without a host sync."""
    d = comm.device
    x = torch.zeros(1 << 22, device=d)
    x.add_(3.0)                                   # producer on the current stream
    w = comm.all_reduce(x, async_op=True)
    w.wait()
    y = x * 2                                     # consumer on the current stream
    torch.cuda.synchronize()
    assert float(y[0]) == 6.0 and float(y[-1]) == 6.0
    assert w.is_completed()


def test_engine_uses_native_comm_at_world1_when_forced(monkeypatch):
    """make_comm picks the native communicator on GPUs only when world > 1 (world 1
    has no traffic); the engine path itself is exercised by tests/test_comm_cpu.py."""
    from kubeflow_controller_amd.parallel.comm import TorchComm, make_comm
    c = make_comm(torch.device("cuda"))
    assert isinstance(c, TorchComm) and c.world == 1
