"""Parameter-server semantics over collectives.

The reference's PS tasks own round-robin-placed variables
(``replica_device_setter``, ``mnist_replica.py:137-141``); workers push
gradients to and pull variables from them over gRPC every step, and the PS
applies Adam with the slots it holds (``:170-184``).  On an 8x MI355X node the
same data movement rides RCCL over xGMI, per gradient bucket
(``parallel/buckets.py``), overlapped with backward:

* **push**  — as soon as a bucket's last gradient lands (backward hook), its
  gradient is widened to fp32 and summed onto its owner(s):
  ``placement="ps"``: ``reduce`` to the rank co-located with the PS task the
  bucket is placed on (round-robin over PS tasks, the ``replica_device_setter``
  rule at bucket granularity); ``placement="sharded"``: ``reduce_scatter`` so
  every worker owns ``1/W`` of every bucket (ZeRO-1 balance).  This IS the
  ``SyncReplicasOptimizer`` accumulator of ``replicas_to_aggregate`` grads
  (K14), folded into the collective.
* **apply** — ONE fused optimizer launch per flat group over the rank's
  compact shard: the fp32 master, the momentum / Adam ``m``/``v`` and the fp32
  gradient exist ONLY for owned elements (per-rank optimizer memory ``1/W``
  with ``sharded``, the PS task's share with ``ps``).
* **pull**  — the updated bf16 weights go back by ``all_gather`` (sharded) /
  ``broadcast`` from the owner (ps), issued asynchronously right after the
  optimizer; a forward pre-hook on each module waits only for the buckets
  holding that module's weights, so the pull of later layers overlaps the
  forward of earlier ones.

Owners are worker ranks (co-located PS, SURVEY §7.3 H1 option a: RCCL refuses
two ranks on one GPU, and the PS replicas get no GPU of their own): PS task
``p`` of ``P`` lives on worker rank ``p * W // P``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .buckets import Bucket, plan_buckets
from .flat import ALIGN, FlatGroup, register_ready_hook


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


def ps_owner_ranks(num_workers: int, num_ps: int) -> List[int]:
    """Worker rank hosting each PS task's variables (spread evenly over the node)."""
    return [p * num_workers // num_ps for p in range(max(1, num_ps))]


# Pull waits per module (default; env KFA_PS_PULL_PER_MODULE=0 turns them off):
# each module's forward pre-hook waits only for the buckets holding its own
# parameters, so the first layers compute while later buckets still arrive.  That
# is only correct if no module reads another module's weight before that module's
# own forward has run, so the model is checked first: a Parameter registered in
# more than one module (tied / shared weights) keeps the single wait-all at the
# start of every forward, and so does a model whose first forward does not show
# every parameter-owning module running its own pre-hook.
PER_MODULE_PULL_WAITS = os.environ.get("KFA_PS_PULL_PER_MODULE", "1") == "1"


def shared_parameters(model: torch.nn.Module) -> List[str]:
    """Names of parameters registered in more than one module (tied weights)."""
    seen: Dict[int, str] = {}
    shared: List[str] = []
    for mname, m in model.named_modules(remove_duplicate=False):
        for pname, p in m.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            if id(p) in seen and seen[id(p)] != full:
                shared.append(f"{seen[id(p)]} = {full}")
            else:
                seen.setdefault(id(p), full)
    return shared


class ShardedGradSync:
    """Bucketed push / owner apply / pull for flat groups (see module docstring)."""

    def __init__(self, groups: Sequence[FlatGroup], process_group=None, *, bucket_mb: float = 32.0,
                 placement: str = "sharded", num_ps: int = 1, reduce_dtype: Optional[torch.dtype] = torch.float32,
                 model: Optional[torch.nn.Module] = None, overlap: bool = True, comm=None):
        from .comm import TorchComm
        if placement not in ("sharded", "ps"):
            raise ValueError(f"placement must be 'sharded' or 'ps', got {placement!r}")
        self.groups = list(groups)
        self.pg = process_group
        self.comm = comm if comm is not None else TorchComm(process_group)  # parallel/comm.py
        self.world = self.comm.world
        self.rank = self.comm.rank
        self.placement = placement if self.world > 1 else "sharded"
        self.num_ps = max(1, num_ps)
        self.owners = ps_owner_ranks(self.world, self.num_ps) if self.placement == "ps" else []
        self.reduce_dtype = reduce_dtype
        self.overlap = overlap and self.world > 1
        unit = ALIGN * (self.world if self.placement == "sharded" else 1)
        self.red_dtypes = [reduce_dtype if (reduce_dtype is not None and self.world > 1) else g.grad.dtype
                           for g in self.groups]
        eb = [torch.empty(0, dtype=d).element_size() for d in self.red_dtypes]
        self.buckets, self._of_param = plan_buckets(self.groups, bucket_mb, unit, eb)
        # ---- ownership + compact shard layout
        self.shard_numel = [0] * len(self.groups)
        per_group_idx = [0] * len(self.groups)
        for b in sorted(self.buckets, key=lambda b: (b.group, b.start)):   # ascending = forward order
            gi = b.group
            if self.placement == "sharded":
                b.owner = -1
                b.shard_off = b.start // self.world
                self.shard_numel[gi] += b.numel // self.world
            else:
                b.owner = self.owners[per_group_idx[gi] % len(self.owners)]
                per_group_idx[gi] += 1
                if b.owner == self.rank:
                    b.shard_off = self.shard_numel[gi]
                    self.shard_numel[gi] += b.numel
        self.w32: List[torch.Tensor] = []
        self.wb: List[Optional[torch.Tensor]] = []
        self.gshard: List[torch.Tensor] = []
        for gi, g in enumerate(self.groups):
            n = self.shard_numel[gi]
            full = g.fp32 if g.master is not None else g.data.float()
            w = torch.empty(n, dtype=torch.float32, device=g.device)
            for b, s, e, off in self._my_chunks(gi):
                w[off:off + (e - s)].copy_(full[s:e])
            self.w32.append(w)
            self.wb.append(torch.empty(n, dtype=g.dtype, device=g.device) if g.dtype != torch.float32 else None)
            self.gshard.append(torch.zeros(n, dtype=self.red_dtypes[gi], device=g.device))
            g.master = None  # the full fp32 master is gone: each rank keeps only what it owns
        self._hooks = []
        if self.overlap:
            for (gi, pi), bs in self._of_param.items():
                p = self.groups[gi].params[pi]
                hook = self._make_hook(bs)
                self._hooks.append(register_ready_hook(p, hook))
        self._pull_hooks = []
        self._stage: Dict[int, torch.Tensor] = {}  # per-bucket reduce-dtype staging (allocated once)
        self._static_mode = "wait-all"
        self._verified = False
        if model is not None and self.world > 1 and PER_MODULE_PULL_WAITS:
            tied = shared_parameters(model)
            if tied:
                self._static_mode = f"wait-all (tied weights: {', '.join(tied[:3])})"
            else:
                self._install_pull_waits(model)
                self._static_mode = None
        self.reset()

    @property
    def pull_mode(self) -> str:
        """What the forward actually waits on: decided by the first forward (see
        ``_root_post``), ``"pending first forward"`` until then."""
        if self._static_mode is not None:
            return self._static_mode
        if not self._verified:
            return "wait-all (pending first forward)"
        n = len(self._root_mods)
        return "per-module" if n == 0 else f"per-module ({n} modules read without their own forward: waited at the root)"

    # ------------------------------------------------------------------ layout
    def _my_chunks(self, gi: int):
        """(bucket, flat start, flat end, shard offset) of every chunk this rank owns in group gi."""
        for b in self.buckets:
            if b.group != gi:
                continue
            if b.owner == -1:
                c = b.numel // self.world
                yield b, b.start + self.rank * c, b.start + (self.rank + 1) * c, b.shard_off
            elif b.owner == self.rank:
                yield b, b.start, b.end, b.shard_off

    def spaces(self):
        """What the fused optimizer updates: this rank's compact shard of each group."""
        from ..ops.optim import OptSpace
        return [OptSpace(g.name, self.w32[gi], self.wb[gi], self.gshard[gi]) for gi, g in enumerate(self.groups)]

    def layout_signature(self) -> str:
        """Identifies the shard layout (checkpoints restore shard files only into the same layout)."""
        parts = [self.placement, str(self.world)]
        for b in self.buckets:
            parts.append(f"{b.group}:{b.start}:{b.end}:{b.owner}")
        return "|".join(parts)

    # ------------------------------------------------------------------ push
    def _make_hook(self, bs: List[Bucket]):
        def hook(_p):
            for b in bs:
                b.pending -= 1
                if b.pending == 0:
                    self._push(b)
                elif b.pending < 0:  # see ddp.GradSync._make_hook
                    raise RuntimeError(f"gradient bucket {b.group}:{b.start}-{b.end} got {b.total - b.pending} "
                                       f"ready notifications for {b.total} tensors (declare tied parameters' "
                                       "uses in _kfa_param_uses)")
        return hook

    def reset(self) -> None:
        for b in self.buckets:
            b.pending = b.total
            b.work = None
            b.tmp = None

    def _staged(self, b: Bucket, view: torch.Tensor, rd: torch.dtype) -> torch.Tensor:
        """``view`` in the reduce dtype: the view itself, or this bucket's staging
        buffer (allocated at the first push, reused every step: the previous step's
        collective on it completed in ``push``)."""
        if view.dtype == rd:
            return view
        buf = self._stage.get(id(b))
        if buf is None:
            buf = self._stage[id(b)] = torch.empty(view.numel(), dtype=rd, device=view.device)
        buf.copy_(view)
        return buf

    def _push(self, b: Bucket) -> None:
        g = self.groups[b.group]
        rd = self.red_dtypes[b.group]
        view = g.grad[b.start:b.end]
        if view.is_cuda:
            from ..ops import streams
            streams.join(view.device)
        if b.owner == -1:
            c = b.numel // self.world
            src = self._staged(b, view, rd)
            out = self.gshard[b.group][b.shard_off:b.shard_off + c]
            b.tmp = src
            b.work = self.comm.reduce_scatter_tensor(out, src, "sum", async_op=True)
        else:
            if b.owner == self.rank:
                buf = self.gshard[b.group][b.shard_off:b.shard_off + b.numel]
                buf.copy_(view)
            else:
                buf = self._staged(b, view, rd)
            b.tmp = buf
            b.work = self.comm.reduce(buf, b.owner, "sum", async_op=True)

    def push(self) -> float:
        """Issue what backward did not, wait for every push; returns the grad scale 1/world."""
        if self.groups and self.groups[0].grad.is_cuda:
            from ..ops import streams
            streams.join(self.groups[0].grad.device)
        if self.world == 1:
            for gi, g in enumerate(self.groups):   # world 1: the shard is the whole group
                self.gshard[gi].copy_(g.grad)
            self.reset()
            return 1.0
        for b in self.buckets:
            if b.work is None:
                self._push(b)
        for b in self.buckets:
            b.work.wait()
        self.reset()
        return 1.0 / self.world

    # ------------------------------------------------------------------ pull
    def pull(self) -> None:
        """Start returning the updated weights to every rank (async; see ``wait_pull``)."""
        if self.world == 1:
            for gi, g in enumerate(self.groups):
                g.data.copy_(self.wb[gi] if self.wb[gi] is not None else self.w32[gi])
            return
        # forward order: the first layers' buckets first
        for b in sorted(self.buckets, key=lambda b: (b.group, b.start)):
            gi = b.group
            g = self.groups[gi]
            src_buf = self.wb[gi] if self.wb[gi] is not None else self.w32[gi]
            out = g.data[b.start:b.end]
            if b.owner == -1:
                c = b.numel // self.world
                b.pull_work = self.comm.all_gather_into_tensor(out, src_buf[b.shard_off:b.shard_off + c],
                                                               async_op=True)
            else:
                if b.owner == self.rank:
                    out.copy_(src_buf[b.shard_off:b.shard_off + b.numel])
                b.pull_work = self.comm.broadcast(out, b.owner, async_op=True)
        if not self._pull_hooks:
            self.wait_pull()

    def wait_pull(self, buckets: Optional[Sequence[Bucket]] = None) -> None:
        for b in (self.buckets if buckets is None else buckets):
            if b.pull_work is not None:
                b.pull_work.wait()
                b.pull_work = None

    def _install_pull_waits(self, model: torch.nn.Module) -> None:
        """Forward pre-hooks: a module waits only for the pulls of the buckets
        holding its own parameters.  That is only safe if every module that owns
        parameters runs its own ``forward`` (a model may read a submodule's
        weight directly), so the root module waits for EVERY pull until one
        forward pass has shown which parameter-owning modules fired their hook.
        Modules that did NOT (their weights are read by another module, e.g.
        ResNet's ``bn_act_dual`` reading bn3 / the downsample BN) have their
        buckets waited at the root from then on; the rest wait in their own hook."""
        by_param = {}
        for gi, g in enumerate(self.groups):
            for pi, p in enumerate(g.params):
                by_param[id(p)] = self._of_param.get((gi, pi), [])
        self._param_modules = set()
        self._mod_buckets: Dict[int, List[Bucket]] = {}
        self._fired = set()
        self._root_mods: set = set()
        self._root_buckets: List[Bucket] = []
        self._verified = False
        for m in model.modules():
            bs = []
            for p in m.parameters(recurse=False):
                for b in by_param.get(id(p), []):
                    if b not in bs:
                        bs.append(b)
            if bs:
                self._param_modules.add(id(m))
                self._mod_buckets[id(m)] = bs
                self._pull_hooks.append(m.register_forward_pre_hook(
                    lambda _m, _i, bs=bs: self._module_wait(_m, bs)))
        self._pull_hooks.append(model.register_forward_pre_hook(lambda _m, _i: self._root_pre()))
        self._pull_hooks.append(model.register_forward_hook(lambda _m, _i, _o: self._root_post()))

    def _module_wait(self, m, bs) -> None:
        self._fired.add(id(m))
        self.wait_pull(bs)

    def _root_pre(self) -> None:
        if not self._verified:
            self.wait_pull()
            self._fired.clear()
        elif self._root_buckets:
            self.wait_pull(self._root_buckets)

    def _root_post(self) -> None:
        if self._verified:
            return
        self._root_mods = self._param_modules - self._fired
        rb: List[Bucket] = []
        for mid in self._root_mods:
            for b in self._mod_buckets[mid]:
                if b not in rb:
                    rb.append(b)
        self._root_buckets = rb
        self._verified = True

    # ------------------------------------------------------------------ checkpoint helpers
    def full_master(self, gi: int) -> torch.Tensor:
        """All ranks: reassemble group ``gi``'s full fp32 master from the owned shards (collective)."""
        g = self.groups[gi]
        full = torch.zeros(g.numel, dtype=torch.float32, device=g.device)
        if self.world == 1:
            full.copy_(self.w32[gi])
            return full
        for b in self.buckets:
            if b.group != gi:
                continue
            out = full[b.start:b.end]
            if b.owner == -1:
                c = b.numel // self.world
                self.comm.all_gather_into_tensor(out, self.w32[gi][b.shard_off:b.shard_off + c])
            else:
                if b.owner == self.rank:
                    out.copy_(self.w32[gi][b.shard_off:b.shard_off + b.numel])
                self.comm.broadcast(out, b.owner)
        return full

    def load_full_master(self, gi: int, full: torch.Tensor) -> None:
        """Take this rank's chunks of a full fp32 master (resume at another world size)."""
        full = full.to(self.w32[gi].device)
        for b, s, e, off in self._my_chunks(gi):
            self.w32[gi][off:off + (e - s)].copy_(full[s:e])

    def remove(self) -> None:
        for h in self._hooks + self._pull_hooks:
            h.remove()
        self._hooks.clear()
        self._pull_hooks.clear()

    def describe(self) -> List[Tuple[str, int, float, int]]:
        return [(self.groups[b.group].name, len(b.params), b.numel * 4 / 2 ** 20, b.owner) for b in self.buckets]
