"""Row-sharded embedding tables with owner-side sparse optimizers — the
"embedding-heavy PS" of BASELINE.json's Wide&Deep config (SURVEY §2.4
"Parameter sharding across PS", §2.6 K6, §7.3 H6).

Reference semantics: ``replica_device_setter`` places each variable on a PS
task (``mnist_replica.py:137-141``); workers pull rows, push gradients, and
the PS applies the optimizer (``:184, :256``).  MI355X design:

* rows are interleaved over ``owners`` ranks (``owner = row % owners``) — with
  PS replicas present the owners are the ranks co-located with the PS tasks
  (SURVEY §7.3 H1 option a), otherwise every rank owns a slice;
* **pull** = each sender's DISTINCT ids (``torch.unique``: ~30 % of the looked-up
  ids at the Criteo-like W&D shape) ``all_to_all``-ed to their owners as local
  row numbers, a HIP gather of the fp32 master rows straight to bf16, an
  ``all_to_all`` back, and an expansion to every lookup;
* **push** = the lookups' gradients pre-summed per distinct id (fp32), one
  ``all_to_all`` of those to the owners (``KFA_EMB_DEDUP=0``: every lookup's id
  and gradient cross, as before), then a
  segment-reduce sparse Adam/SGD (``csrc/kernels/segsparse.hip``): the ids are
  radix-sorted, each row's gradients are summed in fp32 by one workgroup and
  the optimizer is applied once per unique row — no table-sized scratch and
  no per-element atomics (the older scatter-add + atomic-exchange kernels of
  ``csrc/kernels/sparse.hip`` stay behind ``KFA_SPARSE_ATOMIC=1``).  Applied
  during backward, so no dense gradient or optimizer state is ever touched
  for rows outside the batch;
* with one rank (or CPU) the same code runs without collectives;
* the split sizes of the two exchanges come from :meth:`ShardedEmbedding.plan`
  on the host copy of the ids (CPU bincount + a gloo all-to-all of the counts)
  when the batch carries one, so the step never blocks on a device ``.tolist()``.

Parameters marked ``_kfa_sparse`` are skipped by ``split_params`` (they are not
part of the dense flat groups / all-reduce).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import _lib

_P, _L, _I, _F = _lib.P, _lib.L, _lib.I, _lib.F
_lib.register("kfa_scatter_add_rows", [_P, _P, _P, _L, _I, _P])
_lib.register("kfa_sparse_adam", [_P, _P, _P, _P, _P, _L, _I, _F, _F, _F, _F, _F, _F, _F, _F, _P])
_lib.register("kfa_sparse_sgd", [_P, _P, _P, _L, _I, _F, _F, _P])
_lib.register("kfa_embed_fwd", [_P, _P, _P, _P, _P, _P, _I, _P, _L, _I, _L, _P])
_lib.register("kfa_seg_slot_floats", [_L, _I], restype=_L)
_lib.register("kfa_seg_ws_bytes", [_L, _I], restype=_L)
_lib.register("kfa_seg_sparse_apply", [_P, _P, _L, _I, _I, _P, _L, _P, _P, _P, _P, _I] + [_F] * 8 + [_P])
_lib.register("kfa_seg_prepare", [_P, _L, _I, _P, _L, _P])
_lib.register("kfa_seg_prepare_off", [_P, _P, _I, _L, _I, _P, _L, _P])
_lib.register("kfa_seg_apply", [_P, _L, _I, _I, _P, _L, _P, _P, _P, _P, _I] + [_F] * 8 + [_P])
_lib.register("kfa_seg_apply_wd", [_P, _P, _I, _I, _I, _I, _L, _I, _I, _P, _L, _P, _P, _P, _P, _I] + [_F] * 8 + [_P])

_SIDE = {}


def _side_stream(device) -> "torch.cuda.Stream":
    key = str(device)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def _segment_path(n: int, dim: int) -> bool:
    """Sorted segment-reduce update (default) vs the scatter-add + atomic-exchange
    kernels: the segment kernels take 16-byte row vectors (dim % 8 == 0, dim <= 248)."""
    return os.environ.get("KFA_SPARSE_ATOMIC", "0") != "1" and dim % 8 == 0 and dim <= 248 and n < 2 ** 31


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], pg, comm=None) -> None:
    """The id / row / gradient exchange: on the job's communicator when the Engine
    attached one (``ShardedEmbedding.comm``, parallel/comm.py), else torch.distributed."""
    if comm is not None:
        comm.all_to_all_single(out, inp, out_splits, in_splits)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=pg)


class _LookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, emb: "ShardedEmbedding", plan=None):
        ids = ids.reshape(-1)
        n, D = ids.numel(), emb.dim
        comm = emb.world > 1
        inv = order = None
        if comm:
            # local row of each id on its owner; key = owner-major (owner, local row)
            key = (ids % emb.owners) * emb.rows_per_owner + torch.div(ids, emb.owners, rounding_mode="floor")
            if emb.dedup:   # each distinct id crosses the fabric once per sender, both ways
                if plan is not None and len(plan) == 4 and plan[2] is not None:
                    # keys / inverse from the host plan: torch.unique on the device needs its
                    # output size on the host, i.e. a stream drain per lookup
                    ukey, inv = (t.pin_memory().to(ids.device, non_blocking=True) if ids.is_cuda else t
                                 for t in (plan[2], plan[3]))
                else:
                    ukey, inv = torch.unique(key, sorted=True, return_inverse=True)
                send_ids = ukey
            else:
                order = torch.argsort(key, stable=True)
                send_ids = key.index_select(0, order)
            owner_s = torch.div(send_ids, emb.rows_per_owner, rounding_mode="floor")
            send_ids = send_ids - owner_s * emb.rows_per_owner
            if plan is not None:   # split sizes known on the host already: no device sync
                send_l, recv_l = plan[0], plan[1]
            else:                  # derive them on the device (one D2H sync per lookup)
                send = torch.bincount(owner_s, minlength=emb.world)
                recv = torch.empty_like(send)
                _a2a(recv, send, [1] * emb.world, [1] * emb.world, emb.pg, emb.comm)
                send_l, recv_l = send.tolist(), recv.tolist()
            if sum(send_l) != send_ids.numel():
                raise RuntimeError(f"ShardedEmbedding: plan sends {sum(send_l)} ids, lookup has {send_ids.numel()} "
                                   f"({'unique ' if emb.dedup else ''}ids); plan and dedup setting disagree")
            local = torch.empty(sum(recv_l), dtype=ids.dtype, device=ids.device)
            _a2a(local, send_ids, recv_l, send_l, emb.pg, emb.comm)
        else:
            send_l, recv_l = None, None
            local = torch.div(ids, emb.owners, rounding_mode="floor") if emb.owners > 1 else ids
        # the id sort of the sparse update needs no gradient: start it now, beside the dense layers
        ctx.prep = emb.prepare_sparse(local) if ctx.needs_input_grad[1] else None
        rows = emb.gather(local)
        if comm:
            back = torch.empty(sum(send_l), D, dtype=rows.dtype, device=rows.device)
            _a2a(back, rows, send_l, recv_l, emb.pg, emb.comm)
            if inv is not None:
                out = back.index_select(0, inv)
            else:
                out = torch.empty_like(back)
                out.index_copy_(0, order, back)
            isz = ids.element_size()
            emb.exchange_bytes = {"lookups": n, "sent_ids": sum(send_l), "ids": sum(send_l) * isz,
                                  "rows": sum(send_l) * D * rows.element_size(),
                                  "grads": sum(send_l) * D * rows.element_size()}
        else:
            out = rows
        ctx.emb = emb
        e = torch.empty(0, device=ids.device)
        ctx.save_for_backward(local, order if order is not None else e, inv if inv is not None else e)
        ctx.splits = (send_l, recv_l)
        return out

    @staticmethod
    def backward(ctx, dout):
        local, order, inv = ctx.saved_tensors
        emb = ctx.emb
        send_l, recv_l = ctx.splits
        dout = dout.contiguous()
        if emb.world > 1:
            if inv.numel():   # one pre-summed (fp32) gradient per distinct id of this sender
                gu = torch.zeros(sum(send_l), emb.dim, dtype=torch.float32, device=dout.device)
                gu.index_add_(0, inv, dout.float())
                d_send = gu.to(dout.dtype)
            else:
                d_send = dout.index_select(0, order)
            g = torch.empty(local.numel(), emb.dim, dtype=dout.dtype, device=dout.device)
            _a2a(g, d_send, recv_l, send_l, emb.pg, emb.comm)
        else:
            g = dout
        emb.apply_sparse(local, g, prep=ctx.prep)
        ctx.prep = None
        return None, None, None, None


class ShardedEmbedding(nn.Module):
    kfa_sparse_module = True  # split_params leaves the table out of the dense flat groups
    def __init__(self, num_rows: int, dim: int, owners: Optional[int] = None, process_group=None,
                 optimizer: str = "adam", lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, init_std: float = 0.01, seed: int = 0,
                 device=None):
        super().__init__()
        self.pg = process_group
        self.comm = None  # the job's communicator (parallel/comm.py), attached by the Engine
        init = dist.is_initialized()
        self.world = dist.get_world_size(process_group) if init else 1
        self.rank = dist.get_rank(process_group) if init else 0
        self.owners = max(1, min(owners or self.world, self.world))
        self.num_rows, self.dim = num_rows, dim
        self.local_rows = len(range(self.rank, num_rows, self.owners)) if self.rank < self.owners else 0
        self.rows_per_owner = -(-num_rows // self.owners)
        # KFA_EMB_DEDUP=0: every looked-up id (duplicates included) crosses the all-to-alls
        self.dedup = os.environ.get("KFA_EMB_DEDUP", "1") != "0"
        self.exchange_bytes = {}  # last lookup's per-direction all-to-all volume (this rank's sends)
        self.optimizer, self.lr, self.betas, self.eps, self.wd = optimizer, lr, betas, eps, weight_decay
        self.grad_scale = 1.0 / self.world  # data-parallel mean, like the dense groups
        self.t = 0
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self.weight = nn.Parameter(self._init(init_std, seed, dev))
        self.weight._kfa_sparse = True
        self.register_buffer("exp_avg", torch.zeros_like(self.weight) if optimizer == "adam" else None)
        self.register_buffer("exp_avg_sq", torch.zeros_like(self.weight) if optimizer == "adam" else None)

    def _init(self, std: float, seed: int, dev) -> torch.Tensor:
        """World-size independent init: global row r gets the same values on any layout."""
        w = torch.empty(self.local_rows, self.dim, dtype=torch.float32, device=dev)
        if self.local_rows == 0:
            return w
        chunk = 1 << 20
        g = torch.Generator(device=dev)
        for c0 in range(0, self.num_rows, chunk):
            c1 = min(self.num_rows, c0 + chunk)
            g.manual_seed(seed * 1000003 + c0 // chunk)
            blk = torch.randn(c1 - c0, self.dim, generator=g, device=dev) * std
            first = c0 + ((self.rank - c0) % self.owners)       # first owned global row in the chunk
            if first >= c1:
                continue
            rows = torch.arange(first, c1, self.owners, device=dev)
            w[torch.div(rows, self.owners, rounding_mode="floor")] = blk[rows - c0]
        return w

    def extra_repr(self) -> str:
        return (f"rows={self.num_rows}, dim={self.dim}, owners={self.owners}, local_rows={self.local_rows}, "
                f"optimizer={self.optimizer}")

    # ---------------------------------------------------------------- owner-side kernels
    def _check_table(self) -> None:
        """The HIP gather / sparse-optimizer kernels index fp32 [local_rows, dim] rows:
        refuse anything else (e.g. a table some other code cast to bf16) instead of
        letting them address past it."""
        for name, t in (("weight", self.weight), ("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()
                                  or tuple(t.shape) != (self.local_rows, self.dim)):
                raise RuntimeError(f"ShardedEmbedding.{name}: expected contiguous fp32 [{self.local_rows}, "
                                   f"{self.dim}], got {t.dtype} {tuple(t.shape)}")

    def gather(self, local: torch.Tensor) -> torch.Tensor:
        n = local.numel()
        if not self.weight.is_cuda:
            return self.weight.detach().index_select(0, local)
        self._check_table()
        out = torch.empty(n, self.dim, dtype=torch.bfloat16, device=local.device)
        if n:
            _lib.call("kfa_embed_fwd", _lib.ptr(local), _lib.ptr(self.weight), None, None, None, None, 1,
                      _lib.ptr(out), n, self.dim, self.dim, _lib.stream())
        return out

    def _nbits(self) -> int:
        return max(1, (self.local_rows - 1).bit_length())

    @torch.no_grad()
    def prepare_sparse(self, local: torch.Tensor, offsets: Optional[torch.Tensor] = None, F: int = 1):
        """Gradient-independent half of the segment update (radix sort of the ids,
        segment heads) launched on a side stream right after the forward lookup,
        so it runs under the dense layers instead of inside backward.  Returns the
        handle :meth:`apply_sparse` consumes, or None (CPU, atomic path,
        ``KFA_SPARSE_OVERLAP=0``).  ``offsets`` (int64 [F]): ``local`` holds per-table ids of
        F tables stored back to back, row = local[i] + offsets[i % F] (added by the sort's
        key pass, no separate global-row tensor)."""
        n = local.numel()
        if (not self.weight.is_cuda or n == 0 or not _segment_path(n, self.dim)
                or os.environ.get("KFA_SPARSE_OVERLAP", "1") == "0"):
            return None
        nbits = self._nbits()
        ws = torch.empty(_lib.lib().kfa_seg_ws_bytes(n, nbits), dtype=torch.uint8, device=local.device)
        main = torch.cuda.current_stream(local.device)
        side = _side_stream(local.device)
        side.wait_stream(main)
        if offsets is not None:
            if not (offsets.dtype == torch.int64 and offsets.is_contiguous() and offsets.numel() == F and n % F == 0):
                raise ValueError(f"prepare_sparse: offsets {tuple(offsets.shape)} for {n} ids of {F} tables")
            _lib.call("kfa_seg_prepare_off", _lib.ptr(local), _lib.ptr(offsets), F, n, nbits, _lib.ptr(ws), ws.numel(),
                      side.cuda_stream)
            offsets.record_stream(side)
        else:
            _lib.call("kfa_seg_prepare", _lib.ptr(local), n, nbits, _lib.ptr(ws), ws.numel(), side.cuda_stream)
        done = torch.cuda.Event()
        done.record(side)
        ws.record_stream(side)
        local.record_stream(side)
        return ws, nbits, done

    def can_apply_wd(self, local: torch.Tensor, prep) -> bool:
        """:meth:`apply_sparse` can read the row gradients straight from a Wide&Deep MLP
        input gradient (``wd_src``): the GPU segment path with a prepared sort."""
        return prep is not None and self.weight.is_cuda and _segment_path(local.numel(), self.dim)

    @torch.no_grad()
    def apply_sparse(self, local: torch.Tensor, g: Optional[torch.Tensor], prep=None, wd_src=None) -> None:
        """Owner-side sparse update of the rows ``local`` with gradients ``g`` ([n, dim]).
        ``wd_src = (dx, dwide, F, E, Dp)`` (only where :meth:`can_apply_wd`): the row
        gradients are read in place from the Wide&Deep MLP input gradient (row b*F + f =
        [dx[b, Dp + f E : + E] | dwide[b] | 0 ...], ``kfa_seg_apply_wd``) — no [n, dim] copy."""
        self.t += 1
        if local.numel() == 0:
            return
        b1, b2 = self.betas
        if not self.weight.is_cuda:
            self._apply_cpu(local, g.float(), b1, b2)
            return
        self._check_table()
        n, D = local.numel(), self.dim
        st = _lib.stream()
        adam = self.optimizer == "adam"
        c1 = 1.0 / (1.0 - b1 ** self.t) if adam else 1.0
        c2 = 1.0 / (1.0 - b2 ** self.t) if adam else 1.0
        if wd_src is not None:
            if not self.can_apply_wd(local, prep):
                raise ValueError("apply_sparse: wd_src needs the prepared GPU segment path (can_apply_wd)")
            dx, dwide, F, E, Dp = wd_src
            if not (dx.dtype == torch.bfloat16 and dx.is_contiguous() and dx.dim() == 2 and dx.data_ptr() % 16 == 0
                    and dx.shape[0] * F == n and dwide.dtype == torch.float32 and dwide.is_contiguous()
                    and dwide.numel() == dx.shape[0] and D == E + 8 and Dp + F * E <= dx.shape[1]):
                raise ValueError(f"apply_sparse: bad wd_src {tuple(dx.shape)} for {n} rows of {D}")
            ws, nbits, done = prep
            torch.cuda.current_stream().wait_event(done)
            slots = _lib.workspace(_lib.lib().kfa_seg_slot_floats(n, D) * 4, self.weight.device,
                                   f"seg_sparse_slots{id(self)}").view(torch.float32)
            _lib.call("kfa_seg_apply_wd", _lib.ptr(dx), _lib.ptr(dwide), F, E, Dp, dx.shape[1], n, D, nbits,
                      _lib.ptr(ws), ws.numel(), _lib.ptr(slots), _lib.ptr(self.weight), _lib.ptr(self.exp_avg),
                      _lib.ptr(self.exp_avg_sq), 0 if adam else 1, self.lr, b1, b2, self.eps, self.wd, c1, c2,
                      self.grad_scale, st)
            return
        g16 = g.to(torch.bfloat16).contiguous()
        if prep is not None and _segment_path(n, D):
            ws, nbits, done = prep
            torch.cuda.current_stream().wait_event(done)
            slots = _lib.workspace(_lib.lib().kfa_seg_slot_floats(n, D) * 4, self.weight.device,
                                   f"seg_sparse_slots{id(self)}").view(torch.float32)
            _lib.call("kfa_seg_apply", _lib.ptr(g16), n, D, nbits, _lib.ptr(ws), ws.numel(), _lib.ptr(slots),
                      _lib.ptr(self.weight), _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq), 0 if adam else 1,
                      self.lr, b1, b2, self.eps, self.wd, c1, c2, self.grad_scale, st)
            return
        if _segment_path(n, D):
            nbits = self._nbits()
            ws = _lib.workspace(_lib.lib().kfa_seg_ws_bytes(n, nbits), self.weight.device, "seg_sparse_ws")
            slots = _lib.workspace(_lib.lib().kfa_seg_slot_floats(n, D) * 4, self.weight.device,
                                   f"seg_sparse_slots{id(self)}").view(torch.float32)
            _lib.call("kfa_seg_sparse_apply", _lib.ptr(local), _lib.ptr(g16), n, D, nbits, _lib.ptr(ws),
                      ws.numel(), _lib.ptr(slots), _lib.ptr(self.weight), _lib.ptr(self.exp_avg),
                      _lib.ptr(self.exp_avg_sq), 0 if adam else 1, self.lr, b1, b2, self.eps, self.wd, c1, c2,
                      self.grad_scale, st)
            return
        scratch = _lib.workspace(self.local_rows * D * 4, self.weight.device,
                                 f"sparse_scratch{id(self)}").view(torch.float32)
        _lib.call("kfa_scatter_add_rows", _lib.ptr(local), _lib.ptr(g16), _lib.ptr(scratch), n, D, st)
        if adam:
            _lib.call("kfa_sparse_adam", _lib.ptr(local), _lib.ptr(scratch), _lib.ptr(self.weight),
                      _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq), n, D, self.lr, b1, b2,
                      self.eps, self.wd, c1, c2, self.grad_scale, st)
        else:
            _lib.call("kfa_sparse_sgd", _lib.ptr(local), _lib.ptr(scratch), _lib.ptr(self.weight), n, D, self.lr,
                      self.grad_scale, st)

    def _apply_cpu(self, local, g, b1, b2) -> None:
        """Plain-PyTorch reference of the same lazy row update."""
        uniq, inv = torch.unique(local, return_inverse=True)
        gs = torch.zeros(uniq.numel(), self.dim).index_add_(0, inv, g) * self.grad_scale
        w = self.weight.data
        if self.optimizer == "adam":
            nz = gs != 0
            m = self.exp_avg[uniq]
            v = self.exp_avg_sq[uniq]
            m = torch.where(nz, b1 * m + (1 - b1) * gs, m)
            v = torch.where(nz, b2 * v + (1 - b2) * gs * gs, v)
            c1 = 1.0 / (1.0 - b1 ** self.t)
            c2 = 1.0 / (1.0 - b2 ** self.t)
            rows = w[uniq]
            upd = (m * c1) / ((v * c2).sqrt() + self.eps) + self.wd * rows
            w[uniq] = torch.where(nz, rows - self.lr * upd, rows)
            self.exp_avg[uniq] = m
            self.exp_avg_sq[uniq] = v
        else:
            w.index_add_(0, uniq, -self.lr * gs)

    def plan(self, ids_cpu: torch.Tensor):
        """Host-side split sizes for a lookup of ``ids_cpu`` (a CPU tensor, e.g. the
        data loader's batch before its H2D copy): the per-owner counts come from a
        CPU bincount and the receive counts from an all-to-all on a gloo (host)
        group, so the lookup itself never waits for the GPU (``.tolist()`` of a
        device tensor would drain the stream every step).  With dedup the plan also
        carries the sorted distinct keys and the inverse map (CPU tensors), which
        the lookup copies instead of running ``torch.unique`` on the device.

        Returns ``(send_counts, recv_counts, unique_keys | None, inverse | None)``."""
        if self.world == 1:
            return None
        ids_cpu = ids_cpu.reshape(-1).cpu()
        owner = ids_cpu % self.owners
        ukey = inv = None
        if self.dedup:
            key = owner * self.rows_per_owner + torch.div(ids_cpu, self.owners, rounding_mode="floor")
            ukey, inv = torch.unique(key, sorted=True, return_inverse=True)
            owner = torch.div(ukey, self.rows_per_owner, rounding_mode="floor")
        send = torch.bincount(owner, minlength=self.world)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self._meta_group())
        return send.tolist(), recv.tolist(), ukey, inv

    def _meta_group(self):
        if getattr(self, "_meta", None) is None:
            backend = dist.get_backend(self.pg)
            self._meta = self.pg if backend == "gloo" else dist.new_group(backend="gloo")
        return self._meta

    def forward(self, ids: torch.Tensor, plan=None) -> torch.Tensor:
        out = _LookupFn.apply(ids, self.weight, self, plan)
        return out.view(*ids.shape, self.dim)

    def full_table(self) -> torch.Tensor:
        """Gather the whole table to every rank (tests / checkpoint export)."""
        if self.world == 1:
            return self.weight.detach().clone()
        maxr = -(-self.num_rows // self.owners)  # equal-size pieces (gloo needs them)
        mine = torch.zeros(maxr, self.dim, device=self.weight.device)
        mine[:self.local_rows] = self.weight.detach()
        if self.comm is not None:  # the job's communicator (a gloo control group cannot take GPU tensors)
            flat = torch.empty(self.world * maxr, self.dim, device=mine.device)
            self.comm.all_gather_into_tensor(flat, mine)
            parts = list(flat.split(maxr))
        else:
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.pg)
        parts = [p[:len(range(r, self.num_rows, self.owners))] for r, p in enumerate(parts[:self.owners])]
        full = torch.empty(self.num_rows, self.dim, device=self.weight.device)
        for r in range(self.owners):
            full[r::self.owners] = parts[r]
        return full
