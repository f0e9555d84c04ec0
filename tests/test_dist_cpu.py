"""Multi-rank runtime on CPU (gloo): fp32 gradient reduction, sharded /
parameter-server checkpoint-resume, and the ``bench.py --gpus N`` launcher."""
import json
import os
import socket
import subprocess
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


class _Mixed(torch.nn.Module):
    """bf16 weight matrices (fp32 masters) + fp32 biases, like the real models."""

    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(12, 40)
        self.l2 = torch.nn.Linear(40, 5)

    def forward(self, x):
        w1, w2 = self.l1.weight, self.l2.weight
        h = torch.relu(x.to(w1.dtype) @ w1.t() + self.l1.bias.to(w1.dtype))
        return h @ w2.t() + self.l2.bias.to(w2.dtype)


def _model():
    torch.manual_seed(0)
    return _Mixed()


def _data(world, rank):
    g = torch.Generator().manual_seed(1)
    x, y = torch.randn(16, 12, generator=g), torch.randint(0, 5, (16,), generator=g)
    n = 16 // world
    return x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]


def _loss(m, x, y):
    return torch.nn.functional.cross_entropy(m(x).float(), y)


def _engine(rank, world, placement):
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    return Engine(_model(), _loss, optimizer="adam", lr=0.01, compute_dtype=torch.bfloat16, channels_last=False,
                  bucket_mb=0.0005, dist_info=DistInfo(rank=rank, world=world), ps=1 if world > 1 else 0,
                  ps_placement=placement)


def _resume_worker(rank, world, port, phase, placement, ckpt, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.trainer import checkpoint
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(rank, world, placement)
    x, y = _data(world, rank)
    if phase == "ref5":
        for _ in range(5):
            eng.train_step(x, y)
    elif phase == "save3":
        for _ in range(3):
            eng.train_step(x, y)
        eng.save(ckpt, 3, is_chief=False)
        if world > 1:
            dist.barrier()
        if rank == 0:
            checkpoint.write_manifest(ckpt, 3, world)
    elif phase == "resume+2":
        assert eng.restore(ckpt) == 3
        for _ in range(2):
            eng.train_step(x, y)
    elif phase == "resume_w1":
        assert eng.restore(ckpt) == 3
    eng.wait()
    full = [eng.sync.full_master(gi) if eng.sharded else g.fp32.clone() for gi, g in enumerate(eng.groups)]
    if rank == 0:
        torch.save({"sd": {k: v.clone() for k, v in eng.model.state_dict().items()}, "master": full}, out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _run(world, phase, placement, ckpt, out):
    mp.start_processes(_resume_worker, args=(world, _free_port(), phase, placement, ckpt, out), nprocs=world,
                       join=True, start_method="spawn")
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("placement", ["ps", "sharded"])
def test_sharded_resume_is_exact(tmp_path, placement):
    """2 workers + 1 PS, bf16 compute with fp32 masters held only by the owners:
    save at step 3, resume, 2 more steps == 5 uninterrupted steps (bitwise), and a
    1-process resume of the same checkpoint restores the exact fp32 masters."""
    ckpt = str(tmp_path / "ckpt")
    ref5 = _run(2, "ref5", placement, ckpt, str(tmp_path / "ref5.pt"))
    saved = _run(2, "save3", placement, ckpt, str(tmp_path / "save3.pt"))
    resumed = _run(2, "resume+2", placement, ckpt, str(tmp_path / "res.pt"))
    for k, v in ref5["sd"].items():
        assert torch.equal(resumed["sd"][k], v), k
    for a, b in zip(resumed["master"], ref5["master"]):
        assert torch.equal(a, b)
    w1 = _run(1, "resume_w1", placement, ckpt, str(tmp_path / "w1.pt"))
    for k, v in saved["sd"].items():
        assert torch.equal(w1["sd"][k], v), k
    for a, b in zip(w1["master"], saved["master"]):
        n = min(a.numel(), b.numel())  # the groups' tail padding depends on the world size
        assert torch.equal(a[:n], b[:n])
    # the masters differ from the bf16 weights: the resume really restored fp32 state
    assert any(not torch.equal(m.to(torch.bfloat16).float(), m) for m in saved["master"])


def _reduce_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from kubeflow_controller_amd.parallel.ddp import GradSync
    from kubeflow_controller_amd.parallel.flat import split_params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _model()
    groups = split_params(model, torch.bfloat16, pad_to=8 * world)
    x, y = _data(world, rank)
    # this rank's own gradient first, with no sync attached: under overlap the fp32
    # group's buckets are all-reduced IN PLACE while backward is still running, so a
    # clone taken after backward may already hold partial sums
    for g in groups:
        g.zero_grad()
    _loss(model, x, y).backward()
    local = [g.grad.clone() for g in groups]
    sync = GradSync(groups, bucket_mb=0.0005)
    for g in groups:
        g.zero_grad()
    _loss(model, x, y).backward()
    scale = sync.finish()
    torch.save({"local": local, "reduced": [g.opt_grad.clone() for g in groups], "scale": scale,
                "dtypes": [str(g.opt_grad.dtype) for g in groups]}, f"{out}.{rank}")
    dist.destroy_process_group()


def test_bf16_grads_are_summed_in_fp32(tmp_path):
    out = str(tmp_path / "red")
    mp.start_processes(_reduce_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    assert r0["scale"] == 0.5
    assert all(d == "torch.float32" for d in r0["dtypes"])
    for a, b, red in zip(r0["local"], r1["local"], r0["reduced"]):
        torch.testing.assert_close(red, a.float() + b.float(), rtol=0, atol=0)  # exact fp32 sum


def test_bench_launches_ranks_itself():
    """``python bench.py --gpus 2`` (no torchrun, as the driver may call it) starts
    the ranks as a child job and reports n_gpus == 2 (gloo, CPU, tiny model)."""
    env = dict(os.environ, KFA_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--batch", "4", "--image", "32", "--model", "resnet_tiny", "--device",
                        "cpu"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 2 and res["warmup"] == 1
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 8
    assert res["value"] > 0


def test_bench_ps_layout_reports_workers_and_ps():
    """``bench.py --gpus 2 --ps 1``: the '2 workers + 1 PS' BASELINE layout
    (reference examples/tfjob/dist.yml) through the reduce-scatter / owner-apply /
    all-gather path, reported as parallelism "2w1ps"."""
    env = dict(os.environ, KFA_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--ps", "1", "--steps", "2",
                        "--warmup", "1", "--batch", "4", "--image", "32", "--model", "resnet_tiny", "--device",
                        "cpu"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "2w1ps"
    assert res["value"] > 0 and res["config"]["loss"] == res["config"]["loss"]


def test_bench_watchdog_kills_a_hung_rank_and_names_it():
    """One rank stuck before the timed region (the others wait in the barrier):
    the per-rank watchdog dumps every rank's stack and the job exits non-zero
    well inside the watchdog + backstop, with the stuck rank's frame shown."""
    import time
    env = dict(os.environ, KFA_DIST_BACKEND="gloo", OMP_NUM_THREADS="2", KFA_BENCH_HANG_RANK="1")
    env.pop("WORLD_SIZE", None)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--batch", "4", "--image", "32", "--model", "resnet_tiny", "--device",
                        "cpu", "--watchdog", "25"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    dt = time.monotonic() - t0
    assert p.returncode != 0
    assert dt < 25 + 60 + 30, dt
    assert "[rank 1]" in p.stderr and "_test_hang" in p.stderr, p.stderr[-4000:]
    assert "---- rank 1 ----" in p.stderr


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "resnet_tiny",
                        "--device", "cpu"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def _agree_worker(rank, world, port, lockstep, out):
    import torch.distributed as dist
    from kubeflow_controller_amd.ops import conv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    conv.set_lockstep(lockstep)
    # rank 1 would pick differently; only a lockstep job takes rank 0's decision
    got = conv._agree(rank == 0, torch.device("cpu"))
    # the GEMM tuner's multi-way choice (index of the fastest candidate) follows the same rule
    from kubeflow_controller_amd.ops import routes  # every per-shape routing decision (ops/routes.decide)
    pick = routes._agree_index(3 if rank == 0 else 1, torch.device("cpu"))
    out[rank] = (bool(got), pick)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("lockstep", [True, False])
def test_tuner_decision_broadcast_only_in_lockstep_jobs(lockstep):
    """Per-shape tuner choices (conv / dense GEMM) follow rank 0 in a data-parallel
    Engine job; outside one (async-PS workers share their group with PS tasks that
    never run the model) no collective is issued and each rank keeps its own."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_agree_worker, args=(2, _free_port(), lockstep, out), nprocs=2, join=True)
    assert dict(out) == ({0: (True, 3), 1: (True, 3)} if lockstep else {0: (True, 3), 1: (False, 1)})


def _pull_mode_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kubeflow_controller_amd.models.bert import BertConfig, BertForPreTraining, bert_loss, synthetic_mlm_batch
    from kubeflow_controller_amd.models.resnet import resnet_tiny
    from kubeflow_controller_amd.ops.loss import cross_entropy
    from kubeflow_controller_amd.trainer.engine import DistInfo, Engine
    modes = {}
    torch.manual_seed(0)
    r = Engine(resnet_tiny(10), lambda m, x, y: cross_entropy(m(x), y), optimizer="sgd", lr=0.01,
               compute_dtype=torch.bfloat16, channels_last=True, bucket_mb=0.05,
               dist_info=DistInfo(rank=rank, world=world), ps=1, ps_placement="sharded")
    modes["resnet_before"] = r.sync.pull_mode
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    for _ in range(2):
        r.train_step(x, torch.randint(0, 10, (2,)))
    modes["resnet"] = r.sync.pull_mode
    modes["resnet_root"] = len(r.sync._root_buckets)
    cfg = BertConfig.tiny()
    b = Engine(BertForPreTraining(cfg), bert_loss, optimizer="adam", lr=1e-4, compute_dtype=torch.bfloat16,
               channels_last=False, bucket_mb=0.05, dist_info=DistInfo(rank=rank, world=world), ps=1,
               ps_placement="sharded")
    batch = synthetic_mlm_batch(cfg, 2, 16, generator=torch.Generator().manual_seed(rank))
    b.train_step(*batch)
    modes["bert"] = b.sync.pull_mode
    torch.save(modes, f"{out}.{rank}")
    dist.destroy_process_group()


def test_ps_pull_waits_engage_per_module_for_resnet_and_bert(tmp_path):
    """the per-module pull waits must actually engage after the first
    forward.  ResNet's fused ``bn_act_dual`` reads bn3 / downsample-BN weights
    without their own forward: those modules' buckets are waited at the root,
    every other module waits in its own pre-hook (mode "per-module ...")."""
    out = str(tmp_path / "pm")
    mp.start_processes(_pull_mode_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    m = torch.load(f"{out}.0", weights_only=True)
    assert m["resnet_before"].startswith("wait-all (pending"), m
    assert m["resnet"].startswith("per-module"), m
    assert m["bert"].startswith("per-module") or m["bert"].startswith("wait-all (tied"), m
