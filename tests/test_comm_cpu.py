"""First-party communicator (csrc/comm/comm.cpp, parallel/comm.py) vs gloo, on the CPU.

The native layer's host-TCP backend runs the same bootstrap and collective
semantics the RCCL backend drives on GPUs; every collective is compared with
gloo's result for the same inputs (``torch.distributed`` = the test double),
over 3 ranks and several dtypes / reduction ops, plus grouped point-to-point,
uneven all-to-all, and a mismatched-size exchange that must fail (not hang)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.comm import Communicator, TorchComm, default_store
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nat = Communicator.create(default_store(), rank, world, torch.device("cpu"), backend="host", timeout_s=60)
    ref = TorchComm()
    res = {"backend": nat.backend, "bad": []}
    g = torch.Generator().manual_seed(100 + rank)

    def same(name, a, b, exact=True):
        ok = torch.equal(a, b) if exact else torch.allclose(a.float(), b.float(), rtol=1e-6, atol=1e-6)
        if not ok:
            res["bad"].append(f"{name}: max diff {(a.float() - b.float()).abs().max().item()}")

    for dt in (torch.float32, torch.bfloat16, torch.int64, torch.float16, torch.int32, torch.float64):
        # integer-valued data: every summation order gives the same bits in every dtype
        base = torch.randint(-50, 50, (1000,), generator=g)
        for op in ("sum", "max", "min"):
            a, b = base.to(dt).clone(), base.to(dt).clone()
            nat.all_reduce(a, op)
            ref.all_reduce(b, op)
            same(f"all_reduce {dt} {op}", a, b)
        inp = torch.randint(-50, 50, (world * 37,), generator=g).to(dt)
        o1, o2 = torch.empty(37, dtype=dt), torch.empty(37, dtype=dt)
        nat.reduce_scatter_tensor(o1, inp.clone())
        ref.reduce_scatter_tensor(o2, inp.clone())
        same(f"reduce_scatter {dt}", o1, o2)
        src = torch.randint(-50, 50, (53,), generator=g).to(dt)
        o1, o2 = torch.empty(world * 53, dtype=dt), torch.empty(world * 53, dtype=dt)
        nat.all_gather_into_tensor(o1, src)
        ref.all_gather_into_tensor(o2, src)
        same(f"all_gather {dt}", o1, o2)
        for root in range(world):
            a = torch.randint(-50, 50, (29,), generator=g).to(dt)
            b = a.clone()
            nat.broadcast(a, root)
            ref.broadcast(b, root)
            same(f"broadcast {dt} root {root}", a, b)
            a = torch.randint(-50, 50, (31,), generator=g).to(dt)
            b = a.clone()
            nat.reduce(a, root)
            ref.reduce(b, root)
            if rank == root:
                same(f"reduce {dt} root {root}", a, b)
    # fp32 with fractional values: the native sum is in rank order on every rank -> identical bits everywhere
    x = torch.randn(4096, generator=g)
    a = x.clone()
    nat.all_reduce(a)
    allv = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(allv, x)
    expect = allv[0].clone()
    for t in allv[1:]:
        expect += t
    same("all_reduce fp32 rank-order", a, expect)
    # avg
    a, b = x.clone(), x.clone()
    nat.all_reduce(a, "avg")
    ref.all_reduce(b, "sum")
    same("all_reduce avg", a, b / world, exact=False)
    # uneven all-to-all of rows
    in_splits = [(rank + p) % 3 + 1 for p in range(world)]
    out_splits = [(p + rank) % 3 + 1 for p in range(world)]
    inp = torch.randn(sum(in_splits), 5, generator=g)
    o1, o2 = torch.empty(sum(out_splits), 5), torch.empty(sum(out_splits), 5)
    nat.all_to_all_single(o1, inp, out_splits, in_splits)
    ref.all_to_all_single(o2, inp, out_splits, in_splits)
    same("all_to_all_single", o1, o2)
    # ring send / recv in one group (every rank sends to the next, receives from the previous)
    from kubeflow_controller_amd.parallel import comm as C
    msg = torch.full((11,), float(rank))
    got = torch.empty(11)
    C.lib().kfc_group_start(nat._h)
    nat.send(msg, (rank + 1) % world)
    nat.recv(got, (rank - 1) % world)
    C.lib().kfc_group_end(nat._h)
    same("group send/recv", got, torch.full((11,), float((rank - 1) % world)))
    nat.barrier()
    # a size mismatch is reported as an error on the receiver (never a hang or a silent truncation)
    err = ""
    try:
        if rank == 0:
            nat.send(torch.zeros(7), 1)
        elif rank == 1:
            nat.recv(torch.zeros(9), 0)
    except C.CommError as e:
        err = str(e)
    res["mismatch_error"] = err
    torch.save(res, f"{out}.{rank}")
    nat.destroy(abort=True)
    dist.destroy_process_group()


def test_native_host_backend_matches_gloo(tmp_path):
    out = str(tmp_path / "c")
    mp.start_processes(_worker, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    for r in range(3):
        res = torch.load(f"{out}.{r}", weights_only=True)
        assert res["backend"] == "host"
        assert res["bad"] == [], (r, res["bad"])
    assert "size mismatch" in torch.load(f"{out}.1", weights_only=True)["mismatch_error"]


def test_comm_library_surface():
    """The C ABI loads on a machine without GPUs; the RCCL backend resolves librccl
    lazily (present in this image), the dtype table matches ncclDataType_t."""
    sys.path.insert(0, ROOT)
    from kubeflow_controller_amd.parallel import comm as C
    L = C.lib()
    assert [L.kfc_dtype_size(d) if hasattr(L, "kfc_dtype_size") else 0 for d in (0, 6, 7, 9)] in ([1, 2, 4, 2],
                                                                                                   [0, 0, 0, 0])
    assert C._op_code("sum") == 0 and C._op_code(torch.distributed.ReduceOp.MAX) == 2
    h = L.kfc_comm_init(b"nonsense", 1, 0, None, 0, -1, 1000)
    assert not h and b"unknown backend" in L.kfc_last_error()
    h = L.kfc_comm_init(b"host", 1, 0, None, 0, -1, 1000)   # world 1: no sockets at all
    assert h
    t = torch.arange(10, dtype=torch.float32)
    assert L.kfc_all_reduce(h, C._ptr(t), C._ptr(t), 10, 7, 0, None) == 0
    assert torch.equal(t, torch.arange(10, dtype=torch.float32))
    L.kfc_comm_destroy(h)


def _engine_worker(rank, world, port, mode, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KFA_COMM=mode)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine

    class Mlp(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.l1, self.l2 = torch.nn.Linear(12, 40), torch.nn.Linear(40, 5)

        def forward(self, x):
            w1, w2 = self.l1.weight, self.l2.weight
            h = torch.relu(x.to(w1.dtype) @ w1.t() + self.l1.bias.to(w1.dtype))
            return h @ w2.t() + self.l2.bias.to(w2.dtype)

    res = {}
    for ps in (0, 1):
        torch.manual_seed(0)
        m = Mlp()
        eng = Engine(m, lambda mm, x, y: torch.nn.functional.cross_entropy(mm(x).float(), y), optimizer="adam",
                     lr=0.01, compute_dtype=torch.bfloat16, channels_last=False, bucket_mb=0.0005,
                     dist_info=DistInfo(rank=rank, world=world), ps=ps, ps_placement="sharded")
        g = torch.Generator().manual_seed(rank)
        for _ in range(3):
            eng.train_step(torch.randn(8, 12, generator=g), torch.randint(0, 5, (8,), generator=g))
        eng.wait()  # the last step's pull (async) has landed
        res[ps] = {"params": [p.detach().float().clone() for p in m.parameters()], "comm": repr(eng.comm)}
    torch.save(res, f"{out}.{mode}.{rank}")
    dist.destroy_process_group()


def test_engine_native_comm_matches_gloo_training(tmp_path):
    """Three data-parallel training steps (all-reduce, and the sharded PS push /
    apply / pull) give the same weights through the native communicator as through
    gloo (fp32 sums of integer-free data: rank-order vs gloo's order may differ in
    the last bit, hence the tolerance)."""
    out = str(tmp_path / "e")
    for mode in ("native", "torch"):
        mp.start_processes(_engine_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True,
                           start_method="spawn")
    for r in range(2):
        a = torch.load(f"{out}.native.{r}", weights_only=True)
        b = torch.load(f"{out}.torch.{r}", weights_only=True)
        for ps in (0, 1):
            assert a[ps]["comm"].startswith("Communicator(host") and b[ps]["comm"].startswith("TorchComm")
            for x, y in zip(a[ps]["params"], b[ps]["params"]):
                torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_comm_mode_selection(monkeypatch):
    """native only on GPUs with an RCCL process group (a gloo-on-GPU rehearsal keeps
    torch.distributed: RCCL refuses two ranks on one device); KFA_COMM overrides."""
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel import comm as C
    monkeypatch.delenv("KFA_COMM", raising=False)
    assert C.comm_mode(torch.device("cpu")) == "torch"
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda *a: "gloo")
    assert C.comm_mode(torch.device("cuda", 0)) == "torch"
    monkeypatch.setattr(dist, "get_backend", lambda *a: "nccl")
    assert C.comm_mode(torch.device("cuda", 0)) == "native"
    monkeypatch.setenv("KFA_COMM", "torch")
    assert C.comm_mode(torch.device("cuda", 0)) == "torch"
    monkeypatch.setenv("KFA_COMM", "native")
    assert C.comm_mode(torch.device("cpu")) == "native"


def _fallback_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    # the healthy ranks wait this long for the failed one's connection
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KFA_DIST_INIT_TIMEOUT="5")
    os.environ.pop("KFA_COMM", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubeflow_controller_amd.parallel import comm as C
    res = {}
    c = C.make_comm(torch.device("cpu"), mode="native")  # every rank comes up: the native layer is kept
    res["ok"] = repr(c)
    t = torch.full((4,), float(rank + 1))
    c.all_reduce(t, "sum")
    res["ok_sum"] = t.tolist()
    if rank == 1:  # this rank's native bring-up fails: every rank must fall back together
        def broken(*a, **k):
            raise C.CommError("simulated bring-up failure")
        C.Communicator.create = classmethod(lambda cls, *a, **k: broken())
    c2 = C.make_comm(torch.device("cpu"), mode="native")
    res["fallback"] = repr(c2)
    t = torch.full((4,), float(rank + 1))
    c2.all_reduce(t, "sum")
    res["fb_sum"] = t.tolist()
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_make_comm_falls_back_on_every_rank_together(tmp_path):
    """A rank whose native communicator cannot come up makes EVERY rank use
    torch.distributed (decided by one MIN all-reduce over the process group):
    a lone fallback would leave its peers blocked in collectives it never joins."""
    out = str(tmp_path / "f")
    mp.start_processes(_fallback_worker, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    for r in range(3):
        res = torch.load(f"{out}.{r}", weights_only=True)
        assert res["ok"].startswith("Communicator(host"), res
        assert res["fallback"].startswith("TorchComm"), res
        assert res["ok_sum"] == [6.0] * 4 and res["fb_sum"] == [6.0] * 4


def _any_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubeflow_controller_amd.parallel.comm import make_p2p
    p2p = make_p2p(mode="native", timeout_s=60)
    res = {}
    if rank == 0:
        got = []
        buf = torch.zeros(4, dtype=torch.int64)
        for _ in range(2 * (world - 1)):  # two messages from every peer, in whatever order they arrive
            src = p2p.recv_any(buf)
            got.append((src, buf.tolist()))
        res["got"] = got
    else:
        if rank == 1:
            time.sleep(0.3)  # rank 2's messages first
        for k in range(2):
            p2p.send(torch.tensor([rank, k, rank * 10 + k, 7], dtype=torch.int64), 0)
        p2p.destroy()  # a finished peer closes its connections: rank 0 keeps serving the others
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_recv_any_serves_every_peer_in_per_peer_order(tmp_path):
    """kfc_recv_any (the async PS request loop's receive): messages from whichever
    rank sends first, each rank's in its send order, peers that closed skipped."""
    out = str(tmp_path / "any")
    mp.start_processes(_any_worker, args=(3, _free_port(), out), nprocs=3, join=True, start_method="spawn")
    got = torch.load(f"{out}.0", weights_only=True)["got"]
    assert sorted(s for s, _ in got) == [1, 1, 2, 2]
    for r in (1, 2):
        mine = [v for s, v in got if s == r]
        assert mine == [[r, 0, r * 10, 7], [r, 1, r * 10 + 1, 7]]
    assert got[0][0] == 2  # rank 1 started late


def test_one_rccl_communicator_design_decisions(monkeypatch):
    """GPU jobs on the native layer get a gloo default group (control scalars on the
    CPU, no torch RCCL communicator); KFA_COMM=torch keeps nccl; a forced
    KFA_DIST_BACKEND wins (and a forced gloo keeps torch.distributed for the traffic)."""
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel import comm as C
    for v in ("KFA_COMM", "KFA_DIST_BACKEND"):
        monkeypatch.delenv(v, raising=False)
    assert C.dist_backend(use_gpu=True) == "gloo" and C.dist_backend(use_gpu=False) == "gloo"
    monkeypatch.setenv("KFA_COMM", "torch")
    assert C.dist_backend(use_gpu=True) == "nccl"
    monkeypatch.setenv("KFA_DIST_BACKEND", "gloo")
    assert C.dist_backend(use_gpu=True) == "gloo"
    monkeypatch.delenv("KFA_COMM")
    monkeypatch.delenv("KFA_DIST_BACKEND")
    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "get_backend", lambda *a: "gloo")
    monkeypatch.setattr(C, "_CONTROL_ONLY", True)  # what init_default_group sets on a GPU job
    assert C.comm_mode(torch.device("cuda", 0)) == "native"
    assert C.control_device(torch.device("cuda", 0)) == torch.device("cpu")
    monkeypatch.setattr(C, "_CONTROL_ONLY", False)  # KFA_DIST_BACKEND=gloo rehearsal
    assert C.comm_mode(torch.device("cuda", 0)) == "torch"
    monkeypatch.setattr(dist, "get_backend", lambda *a: "nccl")
    assert C.control_device(torch.device("cuda", 0)) == torch.device("cuda", 0)
    assert C.control_device(None) == torch.device("cpu")


def _control_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import datetime
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for v in ("KFA_COMM", "KFA_DIST_BACKEND"):
        os.environ.pop(v, None)
    from kubeflow_controller_amd.parallel import comm as C
    from kubeflow_controller_amd.ops import conv, routes
    # a GPU job's init (gloo needs no device: the "cuda" device only selects the layout)
    be = C.init_default_group(rank, world, torch.device("cuda", 0), datetime.timedelta(seconds=60))
    conv.set_lockstep(True)
    res = {"backend": be, "default": dist.get_backend(), "mode": C.comm_mode(torch.device("cuda", 0)),
           "ctl": str(C.control_device(torch.device("cuda", 0))),
           # the in-step control collectives ride the CPU group: rank 0's pick wins everywhere
           "agree": routes._agree_index(rank + 1, torch.device("cuda", 0)),
           "agree_conv": conv._agree(rank == 0, torch.device("cuda", 0))}
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_gpu_job_default_group_is_control_only_gloo(tmp_path):
    """init_default_group on a GPU job: gloo default group (no torch RCCL
    communicator is ever created while the native layer carries the traffic), the
    native layer selected, control scalars (tuner agreement) on the CPU and
    agreed from rank 0."""
    out = str(tmp_path / "c")
    mp.start_processes(_control_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        res = torch.load(f"{out}.{r}", weights_only=True)
        assert res["backend"] == "gloo" and res["default"] == "gloo", res
        assert res["mode"] == "native" and res["ctl"] == "cpu", res
        assert res["agree"] == 1 and res["agree_conv"] is True, res


def test_parse_rccl_transport(tmp_path):
    """RCCL's INIT/P2P log -> per-peer transport of this rank (bench config.comm)."""
    sys.path.insert(0, ROOT)
    from kubeflow_controller_amd.parallel.comm import parse_rccl_transport
    log = tmp_path / "rccl.log"
    log.write_text(
        "host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 04\n"
        "host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 04\n"
        "host:1:1 [0] NCCL INFO Channel 00/0 : 3[3] -> 0[0] via SHM/direct/direct\n"
        "host:1:1 [0] NCCL INFO Channel 00/0 : 1[1] -> 2[2] via P2P/IPC\n"
        "host:1:1 [0] NCCL INFO Connected all rings\n")
    t = parse_rccl_transport(str(log), 0)
    assert t["via"] == {"P2P/IPC": 2, "SHM/direct/direct": 1}, t
    assert t["peers"] == {"1": "P2P/IPC", "3": "SHM/direct/direct"}, t
    assert parse_rccl_transport(str(tmp_path / "missing.log"), 0) == {"via": "unknown"}
    assert parse_rccl_transport(None, 0) == {"via": "unknown"}


def test_rank0_failure_is_published(monkeypatch):
    """Rank 0 failing before it listens publishes ERR:<why> under the key, so the
    other ranks fail at once instead of waiting out the store timeout."""
    sys.path.insert(0, ROOT)
    import datetime
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel import comm as C
    store = dist.HashStore()
    store.set_timeout(datetime.timedelta(seconds=2))

    def boom():
        raise RuntimeError("comm library failed to build")
    monkeypatch.setattr(C, "lib", boom)
    with pytest.raises(RuntimeError, match="failed to build"):
        C.Communicator.create(store, 0, 2, torch.device("cpu"), key="kfc/t0")
    assert store.get("kfc/t0").decode().startswith("ERR:")
    with pytest.raises(C.CommError, match="rank 0 could not open"):
        C.Communicator.create(store, 1, 2, torch.device("cpu"), key="kfc/t0")


def test_probe_catches_offset_and_order_errors():
    """make_comm's bring-up probe checks every collective the training paths use on
    rank-distinct values element by element (an all-reduce of ones cannot see a
    wrong offset, rank order or op code)."""
    sys.path.insert(0, ROOT)
    from kubeflow_controller_amd.parallel import comm as C

    class Fake:  # a 2-rank job seen from rank 1, with the other rank's inputs simulated
        def __init__(self, bug):
            self.bug = bug

        def reduce_scatter_tensor(self, out, inp, op="sum"):
            n = out.numel()
            base = torch.arange(2 * n, dtype=torch.float32)
            tot = base * 1 + 0.0 + base * 2 + 1000.0   # rank 0's input + rank 1's
            blk = 0 if self.bug == "offset" else 1     # rank 1 owns block 1
            out.copy_(tot[blk * n:(blk + 1) * n])

        def all_gather_into_tensor(self, out, inp):
            n = inp.numel()
            r0 = torch.full((n,), 1.0) + torch.arange(n, dtype=torch.float32)
            parts = [inp, r0] if self.bug == "order" else [r0, inp]
            out.copy_(torch.cat(parts))

        def all_reduce(self, t, op="sum"):
            n = t.numel()
            if op == "max":  # rank 0's probe values: arange
                t.copy_(torch.maximum(t, torch.arange(n, dtype=t.dtype)))
            elif self.bug == "op":  # a wrong op code: max where sum was asked
                t.copy_(torch.maximum(t, (torch.arange(n) % 7 + 1).to(t.dtype)))
            else:
                t.add_((torch.arange(n) % 7 + 1).to(t.dtype))

        def broadcast(self, t, src):
            assert src == 1  # the last rank: this one
            if self.bug == "bcast":  # the root's buffer overwritten by rank 0's
                t.copy_(torch.arange(t.numel(), dtype=t.dtype) * 2)

        def all_to_all_single(self, out, inp, out_splits, in_splits):
            mine = inp[in_splits[0]:in_splits[0] + in_splits[1]]  # the block rank 1 keeps
            peer = torch.full((out_splits[0],), 1.0)            # rank 0 sends 0 * 100 + 1
            out.copy_(torch.cat([mine, peer] if self.bug == "a2a" else [peer, mine])[:out.numel()])
    dev = torch.device("cpu")
    assert C._probe(Fake(None), dev, 2, 1) == "" and C._probe(Fake(None), dev, 2, 1, a2a=True) == ""
    assert "reduce-scatter" in C._probe(Fake("offset"), dev, 2, 1)
    assert "all-gather" in C._probe(Fake("order"), dev, 2, 1)
    assert "all-reduce" in C._probe(Fake("op"), dev, 2, 1)
    assert "broadcast" in C._probe(Fake("bcast"), dev, 2, 1)
    assert C._probe(Fake("a2a"), dev, 2, 1) == ""  # the all-to-all is probed on request only
    assert "all-to-all" in C._probe(Fake("a2a"), dev, 2, 1, a2a=True)
