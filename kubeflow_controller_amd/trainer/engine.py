"""The in-replica training engine: model + flat params + fused optimizer + RCCL grad sync.

Used by ``bench.py`` (headline metric), by the replica runtime
(``trainer/replica.py``, what a TFJob's Worker/Local process runs) and by the
tests.  One process per GPU; ``torch.distributed`` over RCCL (backend "nccl")
when ``world > 1``; gloo on CPU.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..parallel.flat import FlatGroup, split_params


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))

    @property
    def is_chief(self) -> bool:
        return self.rank == 0


def init_distributed(backend: Optional[str] = None, prefer_gpu: bool = True,
                     timeout_s: Optional[float] = None) -> DistInfo:
    """Initialise from torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR/PORT).

    ``KFA_DIST_BACKEND=gloo`` forces gloo even on GPUs: a rehearsal of the
    multi-rank path with several ranks sharing one GPU (RCCL refuses two ranks
    on one device in a communicator).  Otherwise a GPU job's default group is gloo
    for control scalars only and its gradient traffic runs on the first-party RCCL
    communicator (``parallel/comm.py``), so the process holds ONE RCCL
    communicator; ``KFA_COMM=torch`` makes the default group nccl instead.

    ``timeout_s`` (default ``KFA_DIST_INIT_TIMEOUT`` or 300 s) bounds the
    rendezvous and every collective: a rank that never arrives fails the job
    with an error instead of hanging it (RCCL: async error handling on)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL's collectives run concurrently with backward and hold part of the CUs:
        # conv grids of 2x the resident slots let the dispatcher balance around them
        # (a persistent grid waits on its slowest CU).  Costs 0.15 % on one GPU
        # (11,345 -> 11,336 img/s, same box); KFA_CONV_OVERSUB=1 restores persistent.
        os.environ.setdefault("KFA_CONV_OVERSUB", "2")
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        import datetime
        from ..parallel.comm import init_default_group
        t = float(timeout_s if timeout_s is not None else os.environ.get("KFA_DIST_INIT_TIMEOUT", "300"))
        # GPU jobs: a control-only gloo group, the gradients on the native RCCL layer
        # (parallel/comm.py: one RCCL communicator per process); KFA_COMM=torch: nccl
        init_default_group(rank, world, dev, datetime.timedelta(seconds=t), backend=backend)
    return DistInfo(rank, world, local, dev)


class Engine:
    """Owns the flat parameter groups, the gradient sync and the fused optimizer.

    ``ps == 0``: data-parallel all-reduce (``parallel/ddp.py``).  ``ps > 0`` and
    ``world > 1``: parameter-server push/apply/pull (``parallel/ps.py``) with
    ``ps_placement`` ``"ps"`` (variables round-robin on the PS tasks'
    co-located ranks, the reference's ``replica_device_setter``) or
    ``"sharded"`` (every worker owns 1/W).  In both, gradients are summed
    across ranks in ``grad_reduce_dtype`` (fp32 by default) and every
    collective is issued per bucket from backward hooks.

    ``opt_overlap`` (single GPU; env ``KFA_OPT_OVERLAP=1``): the fused optimizer
    runs per gradient bucket on the side stream the moment the bucket's last
    gradient lands, concurrently with the rest of backward, instead of one
    memory-bound pass over every parameter after it (BERT-base Adam: 3.1 GB,
    ~0.59 ms).  Safe because every backward that reads a weight issues that read
    before it reports the weight's gradient ready (``flat.notify_grad_ready`` at
    the end of each HIP Function's backward; autograd's AccumulateGrad after the
    producing node), and the side stream waits for the main stream at each
    bucket; the next step's forward waits for the side stream."""

    def __init__(self, model: torch.nn.Module, loss_fn: Callable, *, optimizer: str = "sgd", lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 compute_dtype=torch.bfloat16, bucket_mb: float = 32.0, dist_info: Optional[DistInfo] = None,
                 channels_last: bool = True, ps: int = 0, ps_placement: str = "ps",
                 grad_reduce_dtype: Optional[torch.dtype] = torch.float32, comm=None,
                 opt_overlap: Optional[bool] = None):
        from ..ops.optim import FusedAdam, FusedSGD
        from ..parallel.ddp import GradSync, broadcast_params

        self.info = dist_info or DistInfo()
        if self.info.world > 1:  # per-shape tuner decisions are broadcast from rank 0 (ops/conv._agree)
            from ..ops import conv as _conv
            _conv.set_lockstep(True)
        self.model = model.to(self.info.device)
        if channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.loss_fn = loss_fn
        # ready-notifications per step of tied parameters (parallel/buckets.py): from
        # each module's map, which copy.deepcopy keeps
        for mod in self.model.modules():
            for pname, uses in getattr(mod, "_kfa_param_uses", {}).items():
                mod.get_parameter(pname)._kfa_uses = int(uses)
        # pad so every group splits evenly into per-rank reduce-scatter shards
        self.groups: List[FlatGroup] = split_params(self.model, compute_dtype, pad_to=8 * max(1, self.info.world))
        # gradient / parameter traffic: the first-party communicator (RCCL on GPUs,
        # parallel/comm.py) unless KFA_COMM=torch; torch.distributed (gloo) on the CPU
        if comm is None:
            from ..parallel.comm import make_comm
            comm = make_comm(self.info.device)
        self.comm = comm
        for m in self.model.modules():  # sparse tables exchange rows on the same communicator
            if getattr(m, "kfa_sparse_module", False) and getattr(m, "world", 1) > 1:
                m.comm = comm
        broadcast_params(self.groups, comm=comm)
        self.sharded = ps > 0 and self.info.world > 1
        if self.sharded:
            from ..parallel.ps import ShardedGradSync
            self.sync = ShardedGradSync(self.groups, bucket_mb=bucket_mb, placement=ps_placement, num_ps=ps,
                                        reduce_dtype=grad_reduce_dtype, model=self.model, comm=comm)
        else:
            self.sync = GradSync(self.groups, bucket_mb=bucket_mb, reduce_dtype=grad_reduce_dtype, comm=comm)
        spaces = self.sync.spaces()
        if optimizer == "sgd":
            self.opt = FusedSGD(spaces, lr=lr, momentum=momentum, weight_decay=weight_decay)
        elif optimizer in ("adam", "adamw"):
            self.opt = FusedAdam(spaces, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        else:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        self.steps = 0
        self._graph = None  # (hipGraph, captured inputs, captured loss) once capture() ran
        if opt_overlap is None:
            opt_overlap = os.environ.get("KFA_OPT_OVERLAP", "0") == "1" and self.info.device.type == "cuda"
        self.opt_overlap = bool(opt_overlap) and self.info.world == 1 and not self.sharded
        self._opt_open = False
        if self.opt_overlap:
            self.sync.on_bucket_ready(self._bucket_update)

    def _bucket_update(self, b) -> None:
        """One gradient bucket complete (host side, during backward): its optimizer
        update on the side stream, after everything queued on the main stream."""
        from ..ops import streams
        dev = self.info.device
        if not self._opt_open:  # the step's count / bias corrections, once, on the main stream
            self.opt.begin_step()
            self._opt_open = True
        if dev.type != "cuda":
            self.opt.update(b.group, b.start, b.end)
            return
        side = streams.side_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self.opt.update(b.group, b.start, b.end)

    def zero_grad(self) -> None:
        for g in self.groups:
            g.zero_grad()

    def train_step(self, *batch) -> torch.Tensor:
        if self._graph is not None:
            return self._replay(batch)
        return self._eager_step(*batch)

    def _eager_step(self, *batch) -> torch.Tensor:
        self._opt_open = False  # (a step whose backward raised never closed its optimizer step)
        self.zero_grad()
        loss = self.loss_fn(self.model, *batch)
        loss.backward()
        if self.sharded:
            self.opt.step(grad_scale=self.sync.push())
            self.sync.pull()   # async; forward pre-hooks wait per bucket
        elif self.opt_overlap:
            from ..ops import streams
            self.sync.finish()  # updates the buckets no gradient reached this step
            if self.info.device.type == "cuda":
                streams.join(self.info.device)
            self._opt_open = False
        else:
            self.opt.step(grad_scale=self.sync.finish())
        self.steps += 1
        return loss.detach()

    # ------------------------------------------------------------------ HIP graph replay
    def graph_ok(self) -> Optional[str]:
        """None if the whole step can be one HIP graph, else why not.

        Every kernel argument is frozen at capture, so what changes per step
        must live in device memory or not change at all: lr / momentum /
        decay are constants, Adam's step count and bias corrections are
        advanced on the device (``kfa_adam_bc``).  A model whose forward takes
        per-step host values (dropout seeds) says so with
        ``graph_capturable = False``.  Collectives stay eager (world > 1): RCCL
        work issued from backward hooks is not replayed through this path.
        The conv tuner and every lazily-created workspace are settled by the
        eager warm-up steps before capture."""
        if self.info.device.type != "cuda":
            return "not on a GPU"
        if self.info.world > 1:
            return "world > 1 (bucket collectives stay eager)"
        if self.opt_overlap:
            return "per-bucket optimizer overlap (opt_overlap) is eager-only"
        if not getattr(self.model, "graph_capturable", True):
            return "the model's forward takes per-step host values (e.g. dropout seeds)"
        if self.opt.step_count == 0:
            return "capture needs one eager step first (momentum init, lazy workspaces)"
        return None

    def capture(self, *batch) -> torch.Tensor:
        """Record one whole training step — zero-grad, forward, loss, backward,
        fused optimizer — as a HIP graph (``torch.cuda.CUDAGraph`` is
        hipGraph on ROCm).  ``train_step`` then copies its batch into the
        captured input buffers (skipped when it passes those same tensors) and
        replays the graph: one launch per step instead of ~470 kernel launches
        through Python, ctypes and autograd."""
        why = self.graph_ok()
        if why is not None:
            raise RuntimeError(f"Engine.capture: {why}")
        static = tuple(batch)
        # warm-up on a side stream first (torch's capture recipe): autograd /
        # allocator state of the capture stream settles before recording.  It is
        # a real training step on `batch`; its loss is returned.
        side = torch.cuda.Stream(self.info.device)
        side.wait_stream(torch.cuda.current_stream(self.info.device))
        with torch.cuda.stream(side):
            warm_loss = self._eager_step(*static)
        torch.cuda.current_stream(self.info.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = self._eager_step(*static)
        self.steps -= 1  # recorded, not executed: each replay counts its step
        self.opt.step_count -= 1
        self._graph = (g, static, loss)
        return warm_loss

    def _replay(self, batch) -> torch.Tensor:
        g, static, loss = self._graph
        for s, b in zip(static, batch):
            if isinstance(s, torch.Tensor) and b is not s:
                s.copy_(b, non_blocking=True)
        g.replay()
        self.opt.step_count += 1
        self.steps += 1
        return loss

    def release_graph(self) -> None:
        self._graph = None

    def wait(self) -> None:
        """Make every rank's compute weights current (after an async pull)."""
        self.sync.wait_pull()

    def num_params(self) -> int:
        return sum(p.numel() for g in self.groups for p in g.params)

    def optimizer_bytes(self) -> int:
        """Bytes of fp32 master + optimizer state + fp32 reduced gradient this rank keeps."""
        n = 0
        for s in self.opt.spaces:
            n += s.w.numel() * 4 if (s.wb is not None or self.sharded) else 0
        for name in ("mom", "m", "v"):
            for b in getattr(self.opt, name, None) or []:
                n += b.numel() * b.element_size() if b is not None else 0
        if self.sharded:
            n += sum(t.numel() * t.element_size() for t in self.sync.gshard)
        else:
            n += sum(g.grad32.numel() * 4 for g in self.groups if g.grad32 is not None)
        return n

    # ------------------------------------------------------------------ checkpoint / resume
    def save(self, model_dir: str, step: int, *, is_chief: Optional[bool] = None, extra: Optional[dict] = None):
        from . import checkpoint
        self.wait()
        full = None
        if self.sharded:  # exact fp32 weights for a resume at another world size (collective)
            full = [self.sync.full_master(gi) for gi in range(len(self.groups))]
        return checkpoint.save(model_dir, step, self.info.rank, self.info.world, self.model, self.groups, self.opt,
                               extra=extra, is_chief=self.info.is_chief if is_chief is None else is_chief,
                               full_masters=full if self.info.is_chief else None, layout=self.layout())

    def restore(self, model_dir: str) -> int:
        from . import checkpoint
        return checkpoint.restore(model_dir, self.info.rank, self.info.world, self.model, self.groups, self.opt,
                                  layout=self.layout(), sync=self.sync if self.sharded else None)

    def comm_info(self) -> dict:
        """What carries this job's gradient traffic (bench JSON ``config.comm``): the
        layer, the default group's backend, RCCL's transport per peer (P2P/IPC =
        xGMI peer access; SHM / NET = a fallback) — None at world 1."""
        c = self.comm
        return {"layer": repr(c) if self.info.world > 1 else None,
                "default_group": dist.get_backend() if dist.is_initialized() else None,
                "transport": c.transport if getattr(c, "native", False) else None}

    def layout(self) -> str:
        return self.sync.layout_signature() if self.sharded else f"allreduce|{self.info.world}"


def synchronize(info: DistInfo) -> None:
    """Device drained, then every rank at the same point (the default group's
    barrier: gloo on the CPU for native-comm GPU jobs, torch's RCCL under
    ``KFA_COMM=torch``)."""
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
        if info.device.type == "cuda":
            torch.cuda.synchronize()


def timed_steps(engine: Engine, batch, steps: int, warmup: int, graph: bool = False) -> Dict[str, float]:
    """W untimed warmup steps, then EXACTLY ``steps`` timed steps bracketed by a
    barrier + device sync on both sides; returns the MAX elapsed over ranks.

    ``graph``: after the warm-up, capture the step as a HIP graph
    (``Engine.capture``) when ``Engine.graph_ok`` allows it, and time replays."""
    for _ in range(warmup):
        engine.train_step(*batch)
    if graph and engine._graph is None and engine.graph_ok() is None:
        synchronize(engine.info)
        engine.capture(*batch)
    synchronize(engine.info)
    cw = getattr(engine.sync, "comm_wait_ms", None)
    if cw is not None:
        cw(reset=True)  # the timed steps' exposed communication only
    t0 = time.perf_counter()
    loss = None
    for _ in range(steps):
        loss = engine.train_step(*batch)
    synchronize(engine.info)
    dt = time.perf_counter() - t0
    from ..parallel.comm import control_device
    t = torch.tensor([dt], dtype=torch.float64, device=control_device(engine.info.device))
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wait = cw() if cw is not None else None
    return {"elapsed": float(t.item()), "loss": float(loss.item()) if loss is not None else float("nan"),
            "comm_wait_ms": round(wait, 4) if wait is not None else None}
