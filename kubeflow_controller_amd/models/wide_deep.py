"""Wide & Deep recommender — BASELINE.json config "Wide&Deep recommender
(embedding-heavy PS), 8 workers + 4 PS co-located on 8×MI355X"
(SURVEY §2.4 parameter sharding, §2.6 K1/K6, §7.3 H6).

* 26 categorical features, Criteo-like cardinalities (22.9 M rows in total),
  one :class:`~kubeflow_controller_amd.parallel.embedding.ShardedEmbedding`
  holding every table back to back (global row = table offset + id), rows
  interleaved over the PS-owner ranks, owner-side sparse Adam.
* Each row is ``embed_dim + 8`` wide: ``embed_dim`` deep features, then the
  wide (linear) weight of that category value in column ``embed_dim`` (the
  remaining 7 columns pad the row to a 16-byte multiple for the HIP gather).
* Deep tower: [13 dense (padded to 16) ‖ 26×embed_dim] → 1024 → 512 → 256 → 1,
  ReLU, GEMM + fused bias/ReLU epilogue kernels; wide part = Σ wide weights +
  linear over the dense features.  Loss: sigmoid cross-entropy.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _lib
from ..ops import transformer as T
from ..parallel.embedding import ShardedEmbedding

_lib.register("kfa_wd_input_fwd", [_lib.P] * 4 + [_lib.I] * 5 + [_lib.P])
_lib.register("kfa_wd_input_bwd", [_lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P])
_lib.register("kfa_wd_gather_fwd", [_lib.P] * 6 + [_lib.I] * 5 + [_lib.P])
_lib.register("kfa_wd_head_blocks", [_lib.I])
_lib.register("kfa_wd_head_fwd_blocks", [_lib.I])
_lib.register("kfa_wd_head_fwd", [_lib.P] * 7 + [_lib.I] * 2 + [_lib.P] * 3 + [_lib.I] * 3 + [_lib.P])
_lib.register("kfa_wd_head_bwd", [_lib.P] * 12 + [_lib.I] * 5 + [_lib.P])


class _WDInputFn(torch.autograd.Function):
    """(rows [B*F, E+8] bf16, dense [B, Dn] fp32) -> (x [B, Dp+F*E] bf16, wide [B] fp32) in
    one HIP pass each way (``csrc/kernels/widedeep.hip``) — the slice / reshape / pad /
    cat / cast chain and its autograd mirror were 16 % of the step.  The dense
    features are zero-padded from Dn to ``Dp`` (default Dn) columns inside the kernel."""

    @staticmethod
    def forward(ctx, rows, dense, B, F, E, Dp=None):
        Dn = dense.shape[1]
        Dp = Dn if Dp is None else Dp
        if not (dense.dtype == torch.float32 and dense.is_contiguous() and Dn <= Dp and Dp % 8 == 0):
            raise ValueError(f"_WDInputFn: dense {tuple(dense.shape)} {dense.dtype} for Dp={Dp}")
        x = torch.empty(B, Dp + F * E, dtype=torch.bfloat16, device=rows.device)
        wide = torch.empty(B, dtype=torch.float32, device=rows.device)
        _lib.call("kfa_wd_input_fwd", _lib.ptr(rows), _lib.ptr(dense), _lib.ptr(x), _lib.ptr(wide), B, F, E, Dp, Dn,
                  _lib.stream())
        ctx.dims = (B, F, E, Dp)
        return x, wide

    @staticmethod
    def backward(ctx, dx, dwide):
        B, F, E, Dp = ctx.dims
        dx = (dx if dx is not None else torch.zeros(B, Dp + F * E, dtype=torch.bfloat16,
                                                    device=dwide.device)).to(torch.bfloat16).contiguous()
        dwide = (dwide if dwide is not None else torch.zeros(B, device=dx.device)).float().contiguous()
        drows = torch.empty(B * F, E + 8, dtype=torch.bfloat16, device=dx.device)
        _lib.call("kfa_wd_input_bwd", _lib.ptr(dx), _lib.ptr(dwide), _lib.ptr(drows), B, F, E, Dp, _lib.stream())
        return drows, None, None, None, None, None


class _WDLookupInputFn(torch.autograd.Function):
    """World-1 lookup + input assembly in one HIP pass (``kfa_wd_gather_fwd``): x rows are
    gathered straight from the fp32 table (bf16-rounded, as the lookup's output) next to
    the zero-padded dense features, wide sums alongside — bit-equal to
    ``ShardedEmbedding`` + :class:`_WDInputFn` without their [B*F, E+8] bf16 rows
    (written once, read once: ~0.13 ms of the 2.0 ms step).  The backward hands the
    rows' gradient to the table's own sparse optimizer as the lookup's backward does
    (``parallel/embedding.py``) — read in place out of dx / dwide by the segment update
    (``kfa_seg_apply_wd``), or materialised by ``kfa_wd_input_bwd`` where that path is off."""

    @staticmethod
    def forward(ctx, ids, offsets, weight, emb, dense, B, F, E, Dp):
        # ids: [B*F] per-table ids; table row = ids[b*F + f] + offsets[f] (added in the kernels)
        Dn = dense.shape[1]
        emb._check_table()
        x = torch.empty(B, Dp + F * E, dtype=torch.bfloat16, device=dense.device)
        wide = torch.empty(B, dtype=torch.float32, device=dense.device)
        # the id sort of the sparse update needs no gradient: start it now, beside the dense layers
        ctx.prep = emb.prepare_sparse(ids, offsets=offsets, F=F) if ctx.needs_input_grad[2] else None
        _lib.call("kfa_wd_gather_fwd", _lib.ptr(ids), _lib.ptr(offsets), _lib.ptr(weight), _lib.ptr(dense), _lib.ptr(x),
                  _lib.ptr(wide), B, F, E, Dp, Dn, _lib.stream())
        ctx.save_for_backward(ids, offsets)
        ctx.emb = emb
        ctx.dims = (B, F, E, Dp)
        return x, wide

    @staticmethod
    def backward(ctx, dx, dwide):
        ids, offsets = ctx.saved_tensors
        B, F, E, Dp = ctx.dims
        gids = ids
        dx = (dx if dx is not None else torch.zeros(B, Dp + F * E, dtype=torch.bfloat16,
                                                    device=gids.device)).to(torch.bfloat16).contiguous()
        dwide = (dwide if dwide is not None else torch.zeros(B, device=gids.device)).float().contiguous()
        emb = ctx.emb
        if FUSED_LOOKUP_BWD and emb.can_apply_wd(gids, ctx.prep):
            # the segment update reads each row's gradient straight out of dx / dwide
            emb.apply_sparse(gids, None, prep=ctx.prep, wd_src=(dx, dwide, F, E, Dp))
        else:
            drows = torch.empty(B * F, E + 8, dtype=torch.bfloat16, device=gids.device)
            _lib.call("kfa_wd_input_bwd", _lib.ptr(dx), _lib.ptr(dwide), _lib.ptr(drows), B, F, E, Dp, _lib.stream())
            # (the prepared sort already holds the global rows; without one, form them here)
            rows = ids if ctx.prep is not None else (ids.view(B, F) + offsets.view(1, F)).reshape(-1)
            emb.apply_sparse(rows, drows, prep=ctx.prep)
        ctx.prep = None
        return None, None, None, None, None, None, None, None, None


def lookup_fusable(emb: ShardedEmbedding, gids: torch.Tensor, E: int) -> bool:
    """:class:`_WDLookupInputFn` applies: one rank holds every row (world 1), the fp32
    table on the GPU with 16-B aligned (E + 8)-wide rows, int64 ids."""
    w = emb.weight
    return (FUSED_INPUT and FUSED_LOOKUP and emb.world == 1 and emb.owners == 1 and w.is_cuda
            and w.dtype == torch.float32 and w.is_contiguous() and emb.dim == E + 8 and E % 8 == 0
            and w.data_ptr() % 16 == 0 and gids.dtype == torch.int64 and gids.is_contiguous())


def _head_weight(t: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    """``t`` flattened as the head kernels read it: its own storage when it already is
    ``dt``, contiguous and 16-B aligned (the flat-buffer views are), else a copy."""
    t = t.detach().reshape(-1)
    if t.dtype == dt and t.is_contiguous() and t.data_ptr() % 16 == 0:
        return t
    return t.to(dt).contiguous()


class _WDHeadFn(torch.autograd.Function):
    """Output head + loss in one HIP pass each way (``csrc/kernels/widedeep.hip``):
    ``z = x . out_w + out_b + wide + dense . wide_dense``, mean sigmoid cross-entropy
    against ``labels``.  Replaces two GEMV-shaped hipBLASLt calls per direction and
    the ATen loss / reduction chain.  Loss and every gradient reduce per-block
    partials in a fixed order (deterministic).

    No glue kernels around it: ``out_w`` / ``wide_dense`` are read in their own dtype
    (bf16 compute copies in the flat buffer, or fp32), ``labels`` as int64 or fp32,
    ``dense`` raw ([B, Dn], Dn <= wide_dense.numel(): the pad columns are zeros), and
    when the three head parameters live in flat gradient buffers the backward ADDS
    their gradients there directly (``parallel/flat.py`` direct-gradient protocol) —
    the fp32 -> bf16 casts and autograd's three accumulate kernels were ~0.04 ms of
    the 2.1 ms W&D step (``profiles/r6_wide_deep_glue.md``)."""

    @staticmethod
    def forward(ctx, x, out_w, out_b, wide, dense, wide_dense, labels):
        B, H = x.shape
        Dn, Dp = dense.shape[1], wide_dense.numel()
        dev = x.device
        wbf = out_w.dtype == torch.bfloat16 and wide_dense.dtype == torch.bfloat16
        wdt = torch.bfloat16 if wbf else torch.float32
        w = _head_weight(out_w, wdt)
        wd = _head_weight(wide_dense, wdt)
        ob = out_b.detach().float().reshape(-1).contiguous()
        yint = labels.dtype == torch.int64
        y = labels.detach().reshape(-1)
        y = (y if (yint or y.dtype == torch.float32) else y.float()).contiguous()
        wide = wide.detach().float().contiguous()
        dense = dense.detach().float().contiguous()
        if Dn > Dp:
            raise ValueError(f"_WDHeadFn: {Dn} dense features for {Dp} wide_dense weights")
        pmy = torch.empty(B, dtype=torch.float32, device=dev)
        part = torch.empty(_lib.lib().kfa_wd_head_fwd_blocks(B), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        _lib.call("kfa_wd_head_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(ob), _lib.ptr(wide), _lib.ptr(dense),
                  _lib.ptr(wd), _lib.ptr(y), int(yint), int(wbf), _lib.ptr(pmy), _lib.ptr(part), _lib.ptr(loss), B, H,
                  Dn, _lib.stream())
        ctx.save_for_backward(x, w, dense, pmy)
        ctx.params = (out_w, out_b, wide_dense)
        ctx.meta = (Dp, wbf)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        from ..parallel.flat import direct_grad_view, notify_grad_ready
        x, w, dense, pmy = ctx.saved_tensors
        out_w, out_b, wide_dense = ctx.params
        Dp, wbf = ctx.meta
        B, H = x.shape
        Dn = dense.shape[1]
        dl = dloss.detach().float().reshape(1).contiguous()
        dx = torch.empty_like(x)
        dwide = torch.empty(B, dtype=torch.float32, device=x.device)
        nb = _lib.lib().kfa_wd_head_blocks(B)
        part = _lib.workspace(4 * nb * (H + Dn + 1), x.device, "wd_head_part")
        views = [direct_grad_view(p) for p in ctx.params]
        wdt = torch.bfloat16 if wbf else torch.float32
        direct = (all(v is not None and v.is_contiguous() for v in views)
                  and views[0].dtype == wdt and views[2].dtype == wdt and views[1].dtype == torch.float32
                  and views[0].numel() == H and views[2].numel() == Dp and views[1].numel() == 1
                  and all(ctx.needs_input_grad[i] for i in (1, 2, 5)))
        grads = None if direct else torch.empty(H + Dp + 1, dtype=torch.float32, device=x.device)
        gw, gb, gwd = views if direct else (None, None, None)
        _lib.call("kfa_wd_head_bwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(dense), _lib.ptr(pmy), _lib.ptr(dl),
                  _lib.ptr(dx), _lib.ptr(dwide), _lib.ptr(part), _lib.ptr(grads), _lib.ptr(gw), _lib.ptr(gwd),
                  _lib.ptr(gb), int(wbf), B, H, Dn, Dp, _lib.stream())
        if direct:
            for p in ctx.params:
                notify_grad_ready(p)
            return dx, None, None, dwide, None, None, None
        return (dx, grads[:H].view(out_w.shape).to(out_w.dtype), grads[H + Dp:].view(out_b.shape).to(out_b.dtype),
                dwide, None, grads[H:H + Dp].view(wide_dense.shape).to(wide_dense.dtype), None)


def head_fusable(x: torch.Tensor, dense: torch.Tensor, dp: int) -> bool:
    return (FUSED_HEAD and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.is_contiguous()
            and x.shape[1] % 8 == 0 and x.shape[1] <= 512 and dense.shape[1] <= dp <= 64 and x.data_ptr() % 16 == 0)


FUSED_HEAD = os.environ.get("KFA_WD_FUSED_HEAD", "1") != "0"  # csrc/kernels/widedeep.hip
FUSED_INPUT = os.environ.get("KFA_WD_FUSED_INPUT", "1") != "0"  # csrc/kernels/widedeep.hip
FUSED_LOOKUP = os.environ.get("KFA_WD_FUSED_LOOKUP", "1") != "0"  # world 1: gather straight into x
# ... and its backward: the table's segment update reads the row gradients out of dx
FUSED_LOOKUP_BWD = os.environ.get("KFA_WD_FUSED_LOOKUP_BWD", "1") != "0"
CRITEO_LIKE = (4_000_000,) * 4 + (1_000_000,) * 6 + (100_000,) * 8 + (10_000,) * 8


@dataclass
class WideDeepConfig:
    num_dense: int = 13
    cardinalities: Tuple[int, ...] = CRITEO_LIKE
    embed_dim: int = 64
    mlp: Tuple[int, ...] = (1024, 512, 256)
    embed_lr: float = 1e-3
    owners: Optional[int] = None       # PS-owner ranks for the tables (None = every rank)

    @classmethod
    def tiny(cls) -> "WideDeepConfig":
        return cls(cardinalities=(1000,) * 4 + (100,) * 4, embed_dim=16, mlp=(64, 32))

    @property
    def row_width(self) -> int:
        return self.embed_dim + 8

    @property
    def dense_pad(self) -> int:
        # (padding the MLP input width to a multiple of 64 so the first layer's K fits
        # the persistent GEMM's k-tiles measured 1 % slower: 25.7 vs 25.9 M ex/s)
        return (self.num_dense + 7) // 8 * 8


class WideDeep(nn.Module):
    # the tables' lazy Adam takes its bias corrections from a host step count, so
    # the step must run eagerly (Engine.graph_ok), not replay a captured graph
    graph_capturable = False

    def __init__(self, cfg: WideDeepConfig, device=None):
        super().__init__()
        self.cfg = cfg
        nf = len(cfg.cardinalities)
        offs = [0]
        for c in cfg.cardinalities[:-1]:
            offs.append(offs[-1] + c)
        self.register_buffer("offsets", torch.tensor(offs, dtype=torch.int64), persistent=False)
        if device is None and torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
        # the tables are created on their final device (22.9 M x 72 fp32 + Adam moments)
        self.tables = ShardedEmbedding(sum(cfg.cardinalities), cfg.row_width, owners=cfg.owners,
                                       lr=cfg.embed_lr, init_std=0.01, device=device)
        dims = [cfg.dense_pad + nf * cfg.embed_dim, *cfg.mlp]
        self.weights = nn.ParameterList()
        self.biases = nn.ParameterList()
        for a, b in zip(dims[:-1], dims[1:]):
            w = nn.Parameter(torch.empty(b, a))
            nn.init.kaiming_uniform_(w, nonlinearity="relu")
            self.weights.append(w)
            self.biases.append(nn.Parameter(torch.zeros(b)))
        self.out_w = nn.Parameter(torch.empty(1, dims[-1]))
        nn.init.normal_(self.out_w, 0.0, dims[-1] ** -0.5)
        self.out_b = nn.Parameter(torch.zeros(1))
        self.wide_dense = nn.Parameter(torch.zeros(1, cfg.dense_pad))

    def _assemble(self, flat_rows, dense, dense32, B, nf, cdt):
        """Looked-up rows [B*nf, E+8] (+ dense) -> (MLP input x, wide sums)."""
        cfg = self.cfg
        if (FUSED_INPUT and flat_rows.is_cuda and flat_rows.dtype == torch.bfloat16 and cdt == torch.bfloat16
                and cfg.embed_dim % 8 == 0 and flat_rows.is_contiguous()):
            return _WDInputFn.apply(flat_rows, dense32, B, nf, cfg.embed_dim, cfg.dense_pad)
        rows = flat_rows.view(B, nf, cfg.row_width)  # [B, nf, E+8]
        deep_emb = rows[:, :, :cfg.embed_dim].reshape(B, nf * cfg.embed_dim)
        wide = rows[:, :, cfg.embed_dim].float().sum(1)
        x = torch.cat([F.pad(dense, (0, cfg.dense_pad - cfg.num_dense)).to(rows.dtype), deep_emb], 1)
        return x, wide

    def forward(self, dense: torch.Tensor, ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        B, nf = ids.shape
        cdt = self.weights[0].dtype
        dense32 = dense.float().contiguous()  # (the fused kernels zero-pad it to dense_pad themselves)
        flat_ids = ids.reshape(-1)
        if cdt == torch.bfloat16 and self.offsets.is_cuda and lookup_fusable(self.tables, flat_ids, cfg.embed_dim):
            # world 1: the lookup gathers straight into the MLP input (global row = id + the
            # table's offset, added inside the gather and the sort's key pass)
            x, wide = _WDLookupInputFn.apply(flat_ids, self.offsets, self.tables.weight, self.tables, dense32, B, nf,
                                             cfg.embed_dim, cfg.dense_pad)
        else:
            gids = (ids + self.offsets.view(1, nf)).reshape(-1)
            x, wide = self._assemble(self.tables(gids, getattr(ids, "_kfa_plan", None)), dense, dense32, B, nf, cdt)
        if x.is_cuda:
            x = x.to(cdt)
            for w, b in zip(self.weights, self.biases):
                x = T.dense(x, w, b, "relu")
        else:
            x = x.float()
            for w, b in zip(self.weights, self.biases):
                x = torch.relu(x @ w.float().t() + b.float())
        if head_fusable(x, dense32, cfg.dense_pad):
            return _WDHeadFn.apply(x, self.out_w, self.out_b, wide, dense32, self.wide_dense, labels)
        dpad = F.pad(dense, (0, cfg.dense_pad - cfg.num_dense))
        deep = (x @ self.out_w.to(x.dtype).t()).float().squeeze(1) + self.out_b.float()
        wide = wide + (dpad.float() @ self.wide_dense.float().t()).squeeze(1)
        return F.binary_cross_entropy_with_logits(deep + wide, labels.float())


def wide_deep_loss(model, *batch):
    return model(*batch)


def prepare_batch(model: "WideDeep", dense: torch.Tensor, ids: torch.Tensor, labels: torch.Tensor, device):
    """Host batch -> device batch whose ids carry the embedding exchange's split
    sizes, computed on the host (``ShardedEmbedding.plan``) before the copy."""
    plan = None
    if model.tables.world > 1:
        gids = ids.cpu() + model.offsets.cpu().view(1, -1)
        plan = model.tables.plan(gids)
    ids_d = ids.to(device)
    if plan is not None:
        ids_d._kfa_plan = plan
    return dense.to(device), ids_d, labels.to(device)


def synthetic_batch(cfg: WideDeepConfig, batch: int, generator=None, device="cpu"):
    """Log-normal dense features, power-law (Zipf-ish) categorical ids, 0/1 labels."""
    g = generator
    dense = torch.log1p(torch.rand(batch, cfg.num_dense, generator=g) * 100.0)
    cols = []
    for c in cfg.cardinalities:
        u = torch.rand(batch, generator=g)
        cols.append(torch.clamp((c ** u).long() - 1, 0, c - 1))      # heavy head, long tail
    ids = torch.stack(cols, 1)
    labels = torch.randint(0, 2, (batch,), generator=g)
    return dense.to(device), ids.to(device), labels.to(device)
