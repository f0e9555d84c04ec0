"""Data-parallel gradient synchronisation over RCCL (xGMI), overlapped with backward.

SURVEY §2.4 "Data parallel: all-reduce (no PS)" and §5.8.  Design for the
MI355X node rather than a DDP clone:

* Gradients already live in flat per-dtype buffers (``parallel/flat.py``), so a
  bucket is a *slice* of that buffer (``parallel/buckets.py``): no gradient
  copy into / out of bucket storage.
* Buckets are cut in reverse parameter order (the order backward produces
  them) at ``bucket_mb`` of reduction dtype (default 32 MB, sized for RCCL's
  channels over the 7 xGMI links, see ``buckets.py``).
* A post-accumulate-grad hook (or a HIP kernel that wrote the gradient straight
  into the flat buffer, ``flat.notify_grad_ready``) counts ready tensors per
  bucket; the bucket's collective is issued the moment its last tensor lands
  (async, on RCCL's stream, ordered after the producing kernels by torch's
  stream semantics).
* **The cross-rank sum runs in fp32** (``reduce_dtype``): a bf16 bucket is
  widened into the group's fp32 reduction buffer by one cast kernel right
  before its all-reduce, and the fused optimizer reads that fp32 buffer.  A
  bf16 ring over 8 ranks rounds every partial sum to 8 significant bits; fp32
  costs 2x the link bytes, which the overlap with backward hides
  (``--grad-reduce bf16`` keeps the old behaviour for A/B).
* The ``1/world`` average is NOT a separate pass: the optimizer kernel takes it
  as ``grad_scale``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .buckets import Bucket, plan_buckets
from .flat import ALIGN, FlatGroup, register_ready_hook


def _join_side_streams(t: torch.Tensor) -> None:
    if t.is_cuda:  # weight-gradient kernels on the side stream wrote into this bucket
        from ..ops import streams
        streams.join(t.device)


class GradSync:
    """``comm``: the communicator the buckets' all-reduces run on (``parallel/comm.py``:
    the first-party RCCL layer on GPUs, ``TorchComm`` = torch.distributed otherwise)."""

    def __init__(self, groups: Sequence[FlatGroup], process_group=None, bucket_mb: float = 32.0,
                 overlap: bool = True, reduce_dtype: Optional[torch.dtype] = torch.float32, comm=None):
        from .comm import TorchComm
        self.groups = list(groups)
        self.pg = process_group
        self.comm = comm if comm is not None else TorchComm(process_group)
        self.world = self.comm.world
        self.overlap = overlap and self.world > 1
        self.reduce_dtype = reduce_dtype
        if self.world > 1 and reduce_dtype is not None:
            for g in self.groups:
                if g.grad.dtype != reduce_dtype:
                    g.grad32 = torch.zeros(g.numel, dtype=reduce_dtype, device=g.device)
        eb = [(g.grad32 if g.grad32 is not None else g.grad).element_size() for g in self.groups]
        self.buckets, self._of_param = plan_buckets(self.groups, bucket_mb, ALIGN, eb)
        self._hooks = []
        self._on_ready = None  # single process: per-bucket callback (Engine's overlapped optimizer)
        # exposed communication per step: compute-stream time from the end of backward
        # to the last bucket's collective (event pairs, read lazily: no host wait)
        self._wait_ev: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []
        self._wait_ms: List[float] = []
        if self.overlap:
            self._install_hooks()
        self.reset()

    def _install_hooks(self) -> None:
        for (gi, pi), bs in self._of_param.items():
            p = self.groups[gi].params[pi]
            hook = self._make_hook(bs)
            # fired either by autograd's AccumulateGrad or by a kernel that wrote
            # the gradient straight into the flat buffer (flat.notify_grad_ready)
            self._hooks.append(register_ready_hook(p, hook))

    def on_bucket_ready(self, cb) -> None:
        """Single process (world == 1, no collective): call ``cb(bucket)`` the moment a
        bucket's last gradient lands during backward, and from ``finish`` for any bucket
        that did not complete (parameters without a gradient this step).  The Engine
        issues that bucket's optimizer update from it (``trainer/engine.py``)."""
        if self.world != 1:
            raise ValueError("on_bucket_ready: world > 1 buckets run their all-reduce")
        self._on_ready = cb
        if not self._hooks:
            self._install_hooks()

    def spaces(self):
        """What the fused optimizer updates: each whole flat group."""
        from ..ops.optim import OptSpace
        return [OptSpace.of_group(g) for g in self.groups]

    def _make_hook(self, bs: List[Bucket]):
        def hook(_p):
            for b in bs:
                b.pending -= 1
                if b.pending == 0:
                    self._launch(b)
                elif b.pending < 0:
                    # a gradient reported ready more often than its bucket counts (an
                    # undeclared tied parameter): the collective already ran without it
                    raise RuntimeError(f"gradient bucket {b.group}:{b.start}-{b.end} got {b.total - b.pending} "
                                       f"ready notifications for {b.total} tensors (declare tied parameters' "
                                       "uses in _kfa_param_uses)")
        return hook

    def reset(self) -> None:
        for b in self.buckets:
            b.pending = b.total
            b.work = None

    def _launch(self, b: Bucket) -> None:
        if self.world == 1:
            if self._on_ready is not None and b.work is None:
                b.work = True
                self._on_ready(b)
            return
        g = self.groups[b.group]
        view = g.grad[b.start:b.end]
        _join_side_streams(view)
        if g.grad32 is not None:
            red = g.grad32[b.start:b.end]
            red.copy_(view)
        else:
            red = view
        b.work = self.comm.all_reduce(red, "sum", async_op=True)

    def finish(self) -> float:
        """Wait for (or issue) every bucket's collective; return the grad scale (1/world)."""
        if self.groups and self.groups[0].grad.is_cuda:
            from ..ops import streams
            streams.join(self.groups[0].grad.device)  # the optimizer reads every weight gradient
        if self.world == 1:
            if self._on_ready is not None:
                for b in self.buckets:
                    self._launch(b)
            self.reset()
            return 1.0
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        timed = self.groups and self.groups[0].grad.is_cuda
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        for b in self.buckets:
            b.work.wait()
        if timed:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._wait_ev.append((e0, e1))
            self._collect(block=False)
        self.reset()
        return 1.0 / self.world

    def _collect(self, block: bool) -> None:
        keep = []
        for e0, e1 in self._wait_ev:
            if block or e1.query():
                if block:
                    e1.synchronize()
                self._wait_ms.append(e0.elapsed_time(e1))
            else:
                keep.append((e0, e1))
        self._wait_ev = keep

    def comm_wait_ms(self, reset: bool = False) -> Optional[float]:
        """Mean per-step time the compute stream waited for the gradient collectives
        after backward had issued its last kernel (the exposed, non-overlapped part of
        the all-reduce), over the steps since the last reset; None at world 1 / CPU."""
        self._collect(block=True)
        v = sum(self._wait_ms) / len(self._wait_ms) if self._wait_ms else None
        if reset:
            self._wait_ms.clear()
        return v

    def pull(self) -> None:
        """No-op: every rank applied the same update to the full weights."""

    def wait_pull(self) -> None:
        """No-op (see ``ps.ShardedGradSync.wait_pull``)."""

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

    def describe(self) -> List[Tuple[str, int, float]]:
        out = []
        for b in self.buckets:
            g = self.groups[b.group]
            eb = (g.grad32 if g.grad32 is not None else g.grad).element_size()
            out.append((g.name, len(b.params), b.numel * eb / 2 ** 20))
        return out


def broadcast_params(groups: Sequence[FlatGroup], src: int = 0, process_group=None, comm=None) -> None:
    """Initial parameter sync from rank ``src`` (owner-initialised
    params broadcast once before the first step)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    for g in groups:
        if comm is not None:
            comm.broadcast(g.fp32, src)
        else:
            dist.broadcast(g.fp32, src, group=process_group)
        if g.master is not None:
            g.data.copy_(g.master)
