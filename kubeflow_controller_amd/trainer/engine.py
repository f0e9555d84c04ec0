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


def init_distributed(backend: Optional[str] = None, prefer_gpu: bool = True) -> DistInfo:
    """Initialise from torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR/PORT).

    ``KFA_DIST_BACKEND=gloo`` forces gloo even on GPUs: a rehearsal of the
    multi-rank path with several ranks sharing one GPU (RCCL refuses two ranks
    on one device in a communicator)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        be = backend or os.environ.get("KFA_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        kw = {"device_id": dev} if (be == "nccl" and use_gpu) else {}
        dist.init_process_group(be, rank=rank, world_size=world, **kw)
    return DistInfo(rank, world, local, dev)


class Engine:
    """Owns the flat parameter groups, the fused optimizer and the grad sync."""

    def __init__(self, model: torch.nn.Module, loss_fn: Callable, *, optimizer: str = "sgd", lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 compute_dtype=torch.bfloat16, bucket_mb: float = 16.0, dist_info: Optional[DistInfo] = None,
                 channels_last: bool = True, ps: int = 0):
        from ..ops.optim import FusedAdam, FusedSGD
        from ..parallel.ddp import GradSync, broadcast_params

        self.info = dist_info or DistInfo()
        self.model = model.to(self.info.device)
        if channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.loss_fn = loss_fn
        # pad so every group splits evenly into per-rank reduce-scatter shards
        self.groups: List[FlatGroup] = split_params(self.model, compute_dtype, pad_to=8 * max(1, self.info.world))
        if optimizer == "sgd":
            self.opt = FusedSGD(self.groups, lr=lr, momentum=momentum, weight_decay=weight_decay)
        elif optimizer in ("adam", "adamw"):
            self.opt = FusedAdam(self.groups, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        else:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        broadcast_params(self.groups)
        # ps > 0: parameter-server layout — shards owned by the
        # ranks, push = reduce-scatter, owner-side fused optimizer, pull = all-gather
        self.sharded = ps > 0 and self.info.world > 1
        if self.sharded:
            from ..parallel.ps import ShardedGradSync
            self.sync = ShardedGradSync(self.groups)
            self.sync.configure(self.opt)
        else:
            self.sync = GradSync(self.groups, bucket_mb=bucket_mb)
        self.steps = 0

    def zero_grad(self) -> None:
        for g in self.groups:
            g.zero_grad()

    def train_step(self, *batch) -> torch.Tensor:
        self.zero_grad()
        loss = self.loss_fn(self.model, *batch)
        loss.backward()
        if self.sharded:
            self.opt.step(grad_scale=self.sync.push())
            self.sync.pull()
        else:
            self.opt.step(grad_scale=self.sync.finish())
        self.steps += 1
        return loss.detach()

    def num_params(self) -> int:
        return sum(p.numel() for g in self.groups for p in g.params)


def synchronize(info: DistInfo) -> None:
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
        if info.device.type == "cuda":
            torch.cuda.synchronize()


def timed_steps(engine: Engine, batch, steps: int, warmup: int) -> Dict[str, float]:
    """W untimed warmup steps, then EXACTLY ``steps`` timed steps bracketed by a
    barrier + device sync on both sides; returns the MAX elapsed over ranks."""
    for _ in range(warmup):
        engine.train_step(*batch)
    synchronize(engine.info)
    t0 = time.perf_counter()
    loss = None
    for _ in range(steps):
        loss = engine.train_step(*batch)
    synchronize(engine.info)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=engine.info.device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"elapsed": float(t.item()), "loss": float(loss.item()) if loss is not None else float("nan")}
