"""Data-parallel correctness on CPU (gloo, world_size 2): bucketed all-reduce
(GradSync) and PS-style reduce-scatter/owner-apply/all-gather (ShardedGradSync)
must reproduce single-process training on the concatenated batch."""
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


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(12, 32), torch.nn.ReLU(), torch.nn.Linear(32, 5))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(16, 12, generator=g), torch.randint(0, 5, (16,), generator=g)


def _train(model, opt, sync, x, y, steps, mode):
    import torch.nn.functional as F
    for _ in range(steps):
        for g in sync.groups:
            g.zero_grad()
        F.cross_entropy(model(x), y).backward()
        if mode != "allreduce":
            scale = sync.push()
            opt.step(grad_scale=scale)
            sync.pull()
        else:
            opt.step(grad_scale=sync.finish())
    sync.wait_pull()


def _make_sync(mode, groups, model, world):
    from kubeflow_controller_amd.parallel.ddp import GradSync
    from kubeflow_controller_amd.parallel.ps import ShardedGradSync
    if mode == "allreduce":
        return GradSync(groups, bucket_mb=0.0005)  # several buckets
    if mode == "sharded":
        return ShardedGradSync(groups, bucket_mb=0.0005, placement="sharded", model=model)
    num_ps = int(mode[2:])  # "ps1", "ps2"
    return ShardedGradSync(groups, bucket_mb=0.0005, placement="ps", num_ps=num_ps, model=model)


def _worker(rank, world, port, mode, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.ops.optim import FusedAdam
    from kubeflow_controller_amd.parallel.ddp import broadcast_params
    from kubeflow_controller_amd.parallel.flat import split_params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _model()
    groups = split_params(model, None, pad_to=8 * world)
    broadcast_params(groups)
    sync = _make_sync(mode, groups, model, world)
    opt = FusedAdam(sync.spaces(), lr=0.01)
    x, y = _data()
    n = x.shape[0] // world
    _train(model, opt, sync, x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n], 5, mode)
    state = {"sd": {k: v.clone() for k, v in model.state_dict().items()},
             "opt_numel": sum(m.numel() for m in opt.m), "buckets": len(sync.buckets)}
    torch.save(state, f"{out}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def _single_process_reference(steps=5):
    from kubeflow_controller_amd.ops.optim import FusedAdam
    from kubeflow_controller_amd.parallel.ddp import GradSync
    from kubeflow_controller_amd.parallel.flat import split_params
    model = _model()
    groups = split_params(model, None)
    sync = GradSync(groups)
    opt = FusedAdam(sync.spaces(), lr=0.01)
    x, y = _data()
    _train(model, opt, sync, x, y, steps, "allreduce")
    return model, groups


@pytest.mark.parametrize("mode", ["allreduce", "sharded", "ps1", "ps2"])
def test_dp_matches_single_process(tmp_path, mode):
    """Every sync mode on 2 gloo ranks (several buckets, parameters straddling
    bucket boundaries, async pulls waited by forward pre-hooks) reproduces one
    process on the concatenated batch, on EVERY rank."""
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True, start_method="spawn")
    model, groups = _single_process_reference()
    full = sum(g.numel for g in groups)
    for r in range(2):
        got = torch.load(f"{out}.{r}", weights_only=True)
        assert got["buckets"] > 2
        for k, v in model.state_dict().items():
            torch.testing.assert_close(got["sd"][k], v, atol=2e-5, rtol=1e-4)
        if mode == "sharded":  # optimizer state only for the owned half
            assert got["opt_numel"] * 2 <= full + 16 * 8
        if mode == "ps1":       # one PS task: its co-located rank 0 owns every variable
            assert (got["opt_numel"] > 0) == (r == 0)


def test_bucket_plan_covers_buffer():
    from kubeflow_controller_amd.parallel.ddp import GradSync
    from kubeflow_controller_amd.parallel.flat import split_params
    model = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
    groups = split_params(model, None)
    sync = GradSync(groups, bucket_mb=0.03)
    for gi, g in enumerate(groups):
        spans = sorted((b.start, b.end) for b in sync.buckets if b.group == gi)
        assert spans[0][0] == 0 and spans[-1][1] == g.numel
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert len(sync.buckets) > 2


def test_ps_assignment():
    from kubeflow_controller_amd.parallel.ps import ps_assignment
    params = [(f"p{i}", torch.empty(s)) for i, s in enumerate([100, 10, 10, 50, 5])]
    rr = ps_assignment(params, 2)
    assert [rr[f"p{i}"] for i in range(5)] == [0, 1, 0, 1, 0]  # replica_device_setter round-robin
    greedy = ps_assignment(params, 2, "greedy")
    load = [sum(p.numel() for n, p in params if greedy[n] == k) for k in range(2)]
    assert max(load) == 100 and min(load) == 75


def _wd_worker(rank, world, port, owners, out, dedup="1"):
    sys.path.insert(0, ROOT)
    os.environ["KFA_EMB_DEDUP"] = dedup
    import torch.distributed as dist
    from kubeflow_controller_amd.models.wide_deep import WideDeep, WideDeepConfig, synthetic_batch, wide_deep_loss
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = WideDeepConfig.tiny()
    cfg.owners = owners
    torch.manual_seed(0)
    m = WideDeep(cfg, device="cpu")
    eng = Engine(m, wide_deep_loss, optimizer="adam", lr=1e-2, compute_dtype=None, channels_last=False,
                 dist_info=DistInfo(rank=rank, world=world))
    dense, ids, labels = synthetic_batch(cfg, 64, torch.Generator().manual_seed(5))
    n = 64 // world
    sl = slice(rank * n, (rank + 1) * n)
    from kubeflow_controller_amd.models.wide_deep import prepare_batch
    for step in range(4):
        if step % 2:   # host-planned split sizes (no device sync) on odd steps, device-derived on even
            eng.train_step(*prepare_batch(m, dense[sl], ids[sl], labels[sl], "cpu"))
        else:
            eng.train_step(dense[sl], ids[sl], labels[sl])
    table = m.tables.full_table()
    if rank == 0:
        sd = {k: v.clone() for k, v in m.state_dict().items() if not k.startswith("tables.")}
        sd["table"] = table
        sd["xbytes"] = torch.tensor([m.tables.exchange_bytes["lookups"], m.tables.exchange_bytes["sent_ids"],
                                     m.tables.exchange_bytes["rows"]])
        torch.save(sd, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("owners,dedup", [(1, "1"), (2, "1"), (2, "0")])
def test_sharded_embedding_ps_matches_single_process(tmp_path, owners, dedup):
    """Wide&Deep with row-sharded tables (all-to-all pull/push, owner-side sparse
    Adam) on 2 ranks == one process on the whole batch — with the deduplicated
    exchange (each sender's distinct ids and pre-summed gradients) and without."""
    from kubeflow_controller_amd.models.wide_deep import WideDeep, WideDeepConfig, synthetic_batch, wide_deep_loss
    from kubeflow_controller_amd.trainer.engine import Engine
    out = str(tmp_path / "wd.pt")
    mp.start_processes(_wd_worker, args=(2, _free_port(), owners, out, dedup), nprocs=2, join=True,
                       start_method="spawn")
    got = torch.load(out, weights_only=True)
    lookups, sent, row_bytes = got.pop("xbytes").tolist()
    if dedup == "1":
        assert sent < lookups, (sent, lookups)   # duplicates never cross the fabric
    else:
        assert sent == lookups
    cfg = WideDeepConfig.tiny()
    torch.manual_seed(0)
    m = WideDeep(cfg, device="cpu")
    eng = Engine(m, wide_deep_loss, optimizer="adam", lr=1e-2, compute_dtype=None, channels_last=False)
    dense, ids, labels = synthetic_batch(cfg, 64, torch.Generator().manual_seed(5))
    for _ in range(4):
        eng.train_step(dense, ids, labels)
    torch.testing.assert_close(got["table"], m.tables.full_table(), atol=1e-5, rtol=1e-4)
    for k, v in m.state_dict().items():
        if not k.startswith("tables."):
            torch.testing.assert_close(got[k], v, atol=1e-5, rtol=1e-4)


def test_bert_tiny_cpu_trains():
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
    from kubeflow_controller_amd.trainer.engine import Engine
    cfg = BertConfig.tiny()
    torch.manual_seed(0)
    m = BertForPreTraining(cfg)
    eng = Engine(m, bert_loss, optimizer="adam", lr=2e-3, compute_dtype=None, channels_last=False)
    batch = synthetic_mlm_batch(cfg, 4, 32, torch.Generator().manual_seed(0))
    losses = [float(eng.train_step(*batch)) for _ in range(15)]
    assert losses[-1] < losses[0] - 0.5, losses


def _async_ps_worker(rank, W, P, port, out, p2p="native"):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.async_ps import AsyncPSClient, AsyncPSServer
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KFA_PS_P2P=p2p)
    dist.init_process_group("gloo", rank=rank, world_size=W + P)
    m = torch.nn.Sequential(torch.nn.Linear(300, 20), torch.nn.Linear(20, 4))
    for p in m.parameters():
        torch.nn.init.constant_(p, 0.5)
    if rank >= W:
        s = AsyncPSServer(list(m.named_parameters()), W, P, rank - W, lr=0.25, optimizer="sgd")
        pushes = s.serve()
        torch.save({"w": s.w, "names": s.names, "pushes": pushes, "step": s.global_step, "p2p": repr(s.p2p)},
                   f"{out}.ps{rank - W}")
        s.close()
    else:
        c = AsyncPSClient(list(m.named_parameters()), W, P)
        steps = []
        for _ in range(7):
            c.pull()
            for p in m.parameters():
                p.grad = torch.full_like(p, float(rank + 1))
            steps.append(c.push())
        c.pull()
        c.done()
        torch.save({"steps": steps, "final": {n: p.detach().clone() for n, p in m.named_parameters()},
                    "p2p": repr(c.p2p)}, f"{out}.w{rank}")
        c.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("p2p", ["native", "torch"])
def test_async_ps_applies_every_push_exactly_once(tmp_path, p2p):
    """Async PS (reference default mode): any-source service loop, round-robin
    placement over 2 PS tasks, every worker push applied once; global step from PS 0.
    Request channel: the first-party host transport (csrc/comm, kfc_recv_any) or gloo."""
    W, P = 3, 2
    out = str(tmp_path / "aps")
    mp.start_processes(_async_ps_worker, args=(W, P, _free_port(), out, p2p), nprocs=W + P, join=True,
                       start_method="spawn")
    want = "P2P(Communicator(host" if p2p == "native" else "P2P(torch.distributed)"
    assert all(torch.load(f"{out}.{r}", weights_only=True)["p2p"].startswith(want)
               for r in ["ps0", "ps1", "w0", "w1", "w2"])
    total = 0.25 * 7 * sum(range(1, W + 1))       # lr * steps * sum of the constant grads
    names = ["0.weight", "0.bias", "1.weight", "1.bias"]
    for k in range(P):
        ps = torch.load(f"{out}.ps{k}", weights_only=True)
        assert ps["names"] == names[k::P]                     # replica_device_setter round-robin
        assert ps["pushes"] == 7 * W
        torch.testing.assert_close(ps["w"], torch.full_like(ps["w"], 0.5 - total))
    steps = sorted(s for w in range(W) for s in torch.load(f"{out}.w{w}", weights_only=True)["steps"])
    assert steps == list(range(1, 7 * W + 1))                  # every push advanced the global step once


def _agg_worker(rank, W, P, N, port, target, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.async_ps import AsyncPSClient, AsyncPSServer
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=W + P)
    m = torch.nn.Sequential(torch.nn.Linear(64, 8), torch.nn.Linear(8, 4))
    for p in m.parameters():
        torch.nn.init.constant_(p, 0.5)
    if rank >= W:
        s = AsyncPSServer(list(m.named_parameters()), W, P, rank - W, lr=0.25, optimizer="sgd", aggregate=N)
        s.serve()
        torch.save({"w": s.w, "step": s.global_step, "applied": s.applied_pushes, "dropped": s.dropped,
                    "sizes": s.update_sizes}, f"{out}.ps{rank - W}")
    else:
        import time
        c = AsyncPSClient(list(m.named_parameters()), W, P)
        step, pushes = 0, 0
        while step < target:
            c.pull()
            for p in m.parameters():
                p.grad = torch.ones_like(p)
            if rank == 0:
                time.sleep(0.01)  # an uneven pace makes some pushes stale
            step = c.push()
            pushes += 1
        c.done()
        torch.save({"pushes": pushes, "dropped": c.pushes_dropped}, f"{out}.w{rank}")
    dist.destroy_process_group()


def test_sync_replicas_aggregates_n_of_w_and_drops_stale(tmp_path):
    """--sync_replicas --replicas_to_aggregate 2 with 3 workers (mnist_replica.py:172-182):
    each update is the MEAN of 2 fresh gradients, pushes computed on an older step
    are dropped, the global step counts updates, and no worker is left waiting."""
    W, P, N, target = 3, 2, 2, 12
    out = str(tmp_path / "agg")
    mp.start_processes(_agg_worker, args=(W, P, N, _free_port(), target, out), nprocs=W + P, join=True,
                       start_method="spawn")
    ws = [torch.load(f"{out}.w{r}", weights_only=True) for r in range(W)]
    total_pushes = sum(w["pushes"] for w in ws)
    for k in range(P):
        ps = torch.load(f"{out}.ps{k}", weights_only=True)
        assert ps["step"] >= target and ps["step"] == len(ps["sizes"])
        assert ps["applied"] + ps["dropped"] == total_pushes          # every push accepted or dropped once
        assert sum(ps["sizes"]) == ps["applied"]
        assert all(1 <= n <= N for n in ps["sizes"]) and ps["sizes"].count(N) >= target - 2
        # all gradients are 1: every update applies a mean of 1 -> w = 0.5 - lr * updates
        torch.testing.assert_close(ps["w"], torch.full_like(ps["w"], 0.5 - 0.25 * ps["step"]))
    ps0 = torch.load(f"{out}.ps0", weights_only=True)
    assert sum(w["dropped"] for w in ws) >= ps0["dropped"] > 0


def test_replicas_to_aggregate_rejected_where_it_cannot_hold():
    """The collective path sums every worker's gradient: N != W is an error, not ignored."""
    from kubeflow_controller_amd.trainer import replica
    base = ["--model", "mnist_mlp", "--sync_replicas", "--replicas_to_aggregate", "1",
            "--worker_hosts=127.0.0.1:1,127.0.0.1:2", "--job_name=worker", "--task_index=0"]
    with pytest.raises(SystemExit, match="collective"):
        replica.main(base + ["--ps_hosts=127.0.0.1:3", "--ps_mode", "collective"])
    with pytest.raises(SystemExit, match="needs PS tasks"):
        replica.main(base + ["--ps_hosts="])
    with pytest.raises(SystemExit, match="1..2"):
        replica.main(base[:4] + ["3"] + base[5:] + ["--ps_hosts=127.0.0.1:3"])


def test_reference_replica_flags_accepted():
    """--existing_servers and --download_only (mnist_replica.py:51-53,76-80) parse;
    --download_only exits 0 once the data set is ready."""
    from kubeflow_controller_amd.trainer import replica
    args = replica.build_parser().parse_args(["--existing_servers", "--download_only=false"])
    assert args.existing_servers is True and args.download_only is False
    assert replica.main(["--download_only", "--model", "mnist_softmax"]) == 0


def test_apply_bit_mask_matches_channels_last_bit_order():
    """ReLU bit masks cover a tensor's channels-last elements, 8 per byte, LSB first."""
    import torch
    from kubeflow_controller_amd.ops.conv import apply_bit_mask
    torch.manual_seed(0)
    t = torch.randn(2, 16, 3, 5).contiguous(memory_format=torch.channels_last)
    keep = torch.rand(2, 3, 5, 16) > 0.5  # NHWC order
    flat = keep.reshape(-1, 8).to(torch.uint8)
    bits = (flat << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    out = apply_bit_mask(t, bits)
    want = t * keep.permute(0, 3, 1, 2)
    assert torch.equal(out, want)


def test_sharded_table_stays_out_of_flat_groups_after_deepcopy():
    """A deep-copied Wide&Deep (tensor attributes do not survive copy.deepcopy) must
    still keep its row-sharded table out of the dense flat groups: cast to the bf16
    compute dtype there, the table's fp32 sparse kernels would write past it."""
    import copy
    from kubeflow_controller_amd.models.wide_deep import WideDeep, WideDeepConfig
    from kubeflow_controller_amd.parallel.flat import split_params
    m = copy.deepcopy(WideDeep(WideDeepConfig.tiny(), device="cpu"))
    groups = split_params(m, torch.bfloat16)
    flat = {id(p) for g in groups for p in g.params}
    assert id(m.tables.weight) not in flat
    assert m.tables.weight.dtype == torch.float32


def test_pull_wait_mode_detects_tied_weights():
    """Per-module pull waits are the default; a Parameter registered in two modules
    (tied weights) keeps the wait-all pull."""
    from kubeflow_controller_amd.parallel.ps import shared_parameters
    a = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    assert shared_parameters(a) == []
    b = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    b[1].weight = b[0].weight
    assert shared_parameters(b) == ["0.weight = 1.weight"]
