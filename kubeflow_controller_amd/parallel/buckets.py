"""Gradient bucket plan shared by the all-reduce (``ddp.GradSync``) and the
parameter-server / sharded (``ps.ShardedGradSync``) synchronisers.

A bucket is a plain ``[start, end)`` slice of a flat group's gradient buffer
(``parallel/flat.py``) — no pack/unpack copies.  Boundaries are cut from the
END of the buffer (backward produces the last parameters' gradients first) at
roughly ``bucket_mb``, snapped to a parameter start and then rounded down to
``unit`` elements.  ``unit = world * ALIGN`` in the sharded modes, so every
bucket splits into ``world`` equal, 16-byte-aligned reduce-scatter chunks; a
parameter may therefore straddle two buckets, and a bucket's collective is
issued once EVERY parameter overlapping it has its gradient.

Sizing for MI355X xGMI: each GPU has 7 point-to-point links of
≈153 GB/s; RCCL runs several rings/channels over them, and a ring moves
``2(n-1)/n · S`` bytes per link.  Buckets of tens of MB keep every channel busy
(a few-MB bucket is latency-bound: ≈10-20 µs per hop) while the last bucket —
the only one exposed after backward — stays ≈0.1-0.3 ms.  The default is 32 MB
of reduction dtype (fp32), i.e. ResNet-50's 102 MB of fp32 gradients in 4
buckets.
"""
from __future__ import annotations

from bisect import bisect_right
from typing import Dict, List, Sequence, Tuple

from .flat import FlatGroup


class Bucket:
    __slots__ = ("index", "group", "start", "end", "params", "pending", "total", "work", "tmp", "owner",
                 "shard_off", "pull_work")

    def __init__(self, index: int, group: int, start: int, end: int):
        self.index = index
        self.group = group
        self.start = start
        self.end = end
        self.params: List[int] = []   # indices into groups[group].params overlapping [start, end)
        self.total = 0                # expected ready-notifications per step
        self.pending = 0
        self.work = None              # in-flight push collective
        self.tmp = None               # staging tensor kept alive until ``work`` completes
        self.owner = -1               # owner rank (PS placement), -1 = every rank owns a chunk
        self.shard_off = 0            # offset of this rank's chunk in its compact shard buffer
        self.pull_work = None         # in-flight pull collective

    @property
    def numel(self) -> int:
        return self.end - self.start

    def __repr__(self) -> str:
        return f"Bucket(g{self.group}[{self.start}:{self.end}], {len(self.params)} params, owner={self.owner})"


def _round_down(n: int, m: int) -> int:
    return n // m * m


def plan_buckets(groups: Sequence[FlatGroup], bucket_mb: float, unit: int, elem_bytes: Sequence[int] = ()
                 ) -> Tuple[List[Bucket], Dict[Tuple[int, int], List[Bucket]]]:
    """Cut every group into buckets; return (buckets in launch order, (group, param) -> buckets).

    ``elem_bytes[g]`` is the byte size of the REDUCTION dtype of group g (the
    cap is in reduction bytes); defaults to the gradient element size."""
    buckets: List[Bucket] = []
    of_param: Dict[Tuple[int, int], List[Bucket]] = {}
    for gi, g in enumerate(groups):
        if g.numel % unit:
            raise ValueError(f"{g}: numel {g.numel} is not a multiple of the bucket unit {unit} (pad_to)")
        eb = elem_bytes[gi] if gi < len(elem_bytes) else g.grad.element_size()
        cap = max(unit, _round_down(int(bucket_mb * (1 << 20)) // eb, unit))
        starts = sorted(set(g.offsets))
        end = g.numel
        mine: List[Bucket] = []
        while end > 0:
            if end - cap <= 0:
                start = 0
            else:
                # the lowest parameter start that keeps the bucket within the cap ...
                i = bisect_right(starts, end - cap - 1)
                cand = starts[i] if i < len(starts) and starts[i] < end else None
                if cand is None:  # ... or, for one parameter larger than the cap, that parameter
                    j = bisect_right(starts, end - 1) - 1
                    cand = starts[j] if j >= 0 else 0
                start = _round_down(cand, unit)
                if start >= end:
                    start = end - unit
            mine.append(Bucket(len(buckets) + len(mine), gi, start, end))
            end = start
        for b in mine:
            for pi, p in enumerate(g.params):
                o, n = g.offsets[pi], p.numel()
                if o < b.end and o + n > b.start:
                    b.params.append(pi)
                    b.total += int(getattr(p, "_kfa_uses", 1))
                    of_param.setdefault((gi, pi), []).append(b)
        buckets.extend(mine)
    for i, b in enumerate(buckets):
        b.index = i
        b.pending = b.total
    return buckets, of_param
