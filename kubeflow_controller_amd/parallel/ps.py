"""Parameter-server semantics over collectives.

The reference's PS tasks own round-robin-placed variables
(``replica_device_setter``, ``mnist_replica.py:137-141``); workers push
gradients to and pull variables from them over gRPC every step.  On an
8x MI355X node the same data movement is:

* push  = ``reduce_scatter`` of the flat gradient buffer: every owner receives
  the SUM of all workers' gradients for the shard it owns (the
  ``SyncReplicasOptimizer`` accumulator of ``replicas_to_aggregate`` grads,
  K14, folded into the collective);
* apply = the fused optimizer kernel on the owner's shard only (fp32 master +
  optimizer state live only on the owner: 1/W of the memory);
* pull  = ``all_gather`` of the updated bf16 compute weights.

Owners are worker ranks (co-located PS, H1 option a): shard ``r`` of every
flat group lives on worker ``r``.  ``ps_assignment`` reproduces the reference's
variable -> PS-task placement (round-robin, or greedy by bytes) for reporting,
checkpoint manifests and the PS coordinator processes.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist

from .flat import ALIGN, FlatGroup


def ps_assignment(params: Sequence[Tuple[str, torch.Tensor]], num_ps: int, strategy: str = "round_robin"
                  ) -> Dict[str, int]:
    """Variable name -> PS task index (``replica_device_setter`` round-robin, or greedy by size)."""
    if num_ps <= 0:
        return {}
    out: Dict[str, int] = {}
    if strategy == "round_robin":
        for i, (n, _) in enumerate(params):
            out[n] = i % num_ps
        return out
    load = [0] * num_ps
    for n, p in sorted(params, key=lambda kv: -kv[1].numel()):
        j = min(range(num_ps), key=lambda k: load[k])
        out[n] = j
        load[j] += p.numel()
    return out


def shard_bounds(numel: int, world: int, rank: int) -> Tuple[int, int]:
    per = numel // world
    assert per % ALIGN == 0, "flat group must be padded to world*ALIGN elements"
    return rank * per, (rank + 1) * per


class ShardedGradSync:
    """Push (reduce-scatter) / owner apply / pull (all-gather) for flat groups.

    Use with a fused optimizer whose ``set_shard`` restricts the update to the
    owned slice; call ``push()`` after backward, ``opt.step(grad_scale=...)``,
    then ``pull()``.
    """

    def __init__(self, groups: Sequence[FlatGroup], process_group=None):
        self.groups = list(groups)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.bounds: List[Tuple[int, int]] = []
        for g in self.groups:
            if g.numel % (self.world * ALIGN):
                raise ValueError(f"{g}: pad the flat group to a multiple of world*{ALIGN} (pad_to)")
            self.bounds.append(shard_bounds(g.numel, self.world, self.rank))

    def configure(self, opt) -> None:
        for gi, (s, e) in enumerate(self.bounds):
            opt.set_shard(gi, s, e)

    def push(self) -> float:
        """Reduce-scatter every group's gradient into the owned shard; returns 1/world."""
        if self.world == 1:
            return 1.0
        works = []
        for g, (s, e) in zip(self.groups, self.bounds):
            out = g.grad[s:e]
            works.append(dist.reduce_scatter_tensor(out, g.grad, op=dist.ReduceOp.SUM, group=self.pg,
                                                    async_op=True))
        for w in works:
            w.wait()
        return 1.0 / self.world

    def pull(self) -> None:
        """All-gather the updated compute weights (bf16 for mixed precision groups)."""
        if self.world == 1:
            return
        works = []
        for g, (s, e) in zip(self.groups, self.bounds):
            works.append(dist.all_gather_into_tensor(g.data, g.data[s:e].clone(), group=self.pg, async_op=True))
        for w in works:
            w.wait()
