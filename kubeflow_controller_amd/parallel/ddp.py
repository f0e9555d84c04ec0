"""Data-parallel gradient synchronisation over RCCL (xGMI), overlapped with backward.

SURVEY §2.4 "Data parallel: all-reduce (no PS)" and §5.8.  Design for the
MI355X node rather than a DDP clone:

* Gradients already live in flat per-dtype buffers (``parallel/flat.py``), so a
  bucket is a *slice* of that buffer: no gradient copy into / out of bucket
  storage.
* Buckets are cut in reverse parameter order (the order backward produces
  them) at ``bucket_mb`` (default 16 MB: large enough to light up RCCL's
  channels across the 7 xGMI links, small enough that the last bucket's
  exposed all-reduce after backward stays ~0.1 ms).
* A post-accumulate-grad hook counts ready tensors per bucket; the bucket's
  collective is issued the moment its last tensor lands (async, on RCCL's
  stream, ordered after the producing kernels by torch's stream semantics).
* The ``1/world`` average is NOT a separate pass: the optimizer kernel takes it
  as ``grad_scale``.
* ``mode="allreduce"`` (pure DP) or ``mode="reduce_scatter"`` (ZeRO-1 /
  parameter-server shards: each rank only receives — and only updates — the
  shard it owns, then ``all_gather`` refreshes the compute weights; see
  ``parallel/ps.py``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .flat import FlatGroup, set_ready_callback


class _Bucket:
    __slots__ = ("group", "start", "end", "params", "pending", "work")

    def __init__(self, group: int, start: int, end: int):
        self.group = group
        self.start = start
        self.end = end
        self.params: List[int] = []
        self.pending = 0
        self.work = None


class GradSync:
    def __init__(self, groups: Sequence[FlatGroup], process_group=None, bucket_mb: float = 16.0,
                 overlap: bool = True):
        self.groups = list(groups)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.overlap = overlap and self.world > 1
        self.buckets: List[_Bucket] = []
        self._hooks = []
        self._tensor_bucket = {}
        for gi, g in enumerate(self.groups):
            cap = max(int(bucket_mb * (1 << 20)) // g.grad.element_size(), 8)
            cur: Optional[_Bucket] = None
            # walk params from last to first (backward order)
            order = list(range(len(g.params)))[::-1]
            for pi in order:
                s, e = g.offsets[pi], g.offsets[pi] + g.params[pi].numel()
                if cur is None or (cur.end - s) > cap:
                    end = g.numel if cur is None else cur.start
                    cur = _Bucket(gi, s, end)
                    self.buckets.append(cur)
                cur.start = s
                cur.params.append(pi)
                self._tensor_bucket[(gi, pi)] = cur
            if cur is not None:
                cur.start = 0
        if self.overlap:
            for (gi, pi), b in self._tensor_bucket.items():
                p = self.groups[gi].params[pi]
                hook = self._make_hook(b)
                # fired either by autograd's AccumulateGrad or by a kernel that wrote
                # the gradient straight into the flat buffer (flat.notify_grad_ready)
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))
                set_ready_callback(p, hook)
        self.reset()

    def _make_hook(self, b: _Bucket):
        def hook(_p):
            b.pending -= 1
            if b.pending == 0:
                self._launch(b)
        return hook

    def reset(self) -> None:
        for b in self.buckets:
            # a tied parameter written by several direct-gradient kernels per step
            # (e.g. BERT's word embedding: lookup + MLM decoder) declares _kfa_uses
            b.pending = sum(getattr(self.groups[b.group].params[pi], "_kfa_uses", 1) for pi in b.params)
            b.work = None

    def _launch(self, b: _Bucket) -> None:
        view = self.groups[b.group].grad[b.start:b.end]
        if view.is_cuda:  # weight-gradient kernels on the side stream wrote into this bucket
            from ..ops import streams
            streams.join(view.device)
        b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def finish(self) -> float:
        """Wait for (or issue) every bucket's collective; return the grad scale (1/world)."""
        if self.world == 1:
            self.reset()
            return 1.0
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
        self.reset()
        return 1.0 / self.world

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

    def describe(self) -> List[Tuple[str, int, float]]:
        return [(self.groups[b.group].name, len(b.params),
                 (b.end - b.start) * self.groups[b.group].grad.element_size() / 2 ** 20) for b in self.buckets]


def broadcast_params(groups: Sequence[FlatGroup], src: int = 0, process_group=None) -> None:
    """Initial parameter sync from rank ``src`` (owner-initialised
    params broadcast once before the first step)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    for g in groups:
        dist.broadcast(g.fp32, src, group=process_group)
        if g.master is not None:
            g.data.copy_(g.master)
