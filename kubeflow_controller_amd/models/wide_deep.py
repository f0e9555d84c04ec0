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

_lib.register("kfa_wd_input_fwd", [_lib.P, _lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P])
_lib.register("kfa_wd_input_bwd", [_lib.P, _lib.P, _lib.P, _lib.I, _lib.I, _lib.I, _lib.I, _lib.P])
_lib.register("kfa_wd_head_blocks", [_lib.I])
_lib.register("kfa_wd_head_fwd", [_lib.P] * 10 + [_lib.I] * 3 + [_lib.P])
_lib.register("kfa_wd_head_bwd", [_lib.P] * 9 + [_lib.I] * 3 + [_lib.P])


class _WDInputFn(torch.autograd.Function):
    """(rows [B*F, E+8] bf16, dense_pad [B, Dp] fp32) -> (x [B, Dp+F*E] bf16, wide [B] fp32) in
    one HIP pass each way (``csrc/kernels/widedeep.hip``) — the slice / reshape / pad /
    cat / cast chain and its autograd mirror were 16 % of the step."""

    @staticmethod
    def forward(ctx, rows, dense_pad, B, F, E):
        Dp = dense_pad.shape[1]
        x = torch.empty(B, Dp + F * E, dtype=torch.bfloat16, device=rows.device)
        wide = torch.empty(B, dtype=torch.float32, device=rows.device)
        _lib.call("kfa_wd_input_fwd", _lib.ptr(rows), _lib.ptr(dense_pad), _lib.ptr(x), _lib.ptr(wide), B, F, E, Dp,
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
        return drows, None, None, None, None


class _WDHeadFn(torch.autograd.Function):
    """Output head + loss in one HIP pass each way (``csrc/kernels/widedeep.hip``):
    ``z = x . out_w + out_b + wide + dpad . wide_dense``, mean sigmoid cross-entropy
    against ``labels``.  Replaces two GEMV-shaped hipBLASLt calls per direction and
    the ATen loss / reduction chain.  Loss and every gradient reduce per-block
    partials in a fixed order (deterministic)."""

    @staticmethod
    def forward(ctx, x, out_w, out_b, wide, dpad, wide_dense, labels):
        B, H = x.shape
        Dp = dpad.shape[1]
        dev = x.device
        w = out_w.detach().float().reshape(-1).contiguous()
        ob = out_b.detach().float().reshape(-1).contiguous()
        wd = wide_dense.detach().float().reshape(-1).contiguous()
        y = labels.detach().float().reshape(-1).contiguous()
        wide = wide.detach().float().contiguous()
        pmy = torch.empty(B, dtype=torch.float32, device=dev)
        part = torch.empty(_lib.lib().kfa_wd_head_blocks(B), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        _lib.call("kfa_wd_head_fwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(ob), _lib.ptr(wide), _lib.ptr(dpad), _lib.ptr(wd),
                  _lib.ptr(y), _lib.ptr(pmy), _lib.ptr(part), _lib.ptr(loss), B, H, Dp, _lib.stream())
        ctx.save_for_backward(x, w, dpad, pmy)
        ctx.meta = (out_w.shape, out_w.dtype, out_b.shape, out_b.dtype, wide_dense.shape, wide_dense.dtype)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        x, w, dpad, pmy = ctx.saved_tensors
        wshape, wdt, bshape, bdt, wdshape, wddt = ctx.meta
        B, H = x.shape
        Dp = dpad.shape[1]
        dl = dloss.detach().float().reshape(1).contiguous()
        dx = torch.empty_like(x)
        dwide = torch.empty(B, dtype=torch.float32, device=x.device)
        nb = _lib.lib().kfa_wd_head_blocks(B)
        part = _lib.workspace(4 * nb * (H + Dp + 1), x.device, "wd_head_part")
        grads = torch.empty(H + Dp + 1, dtype=torch.float32, device=x.device)
        _lib.call("kfa_wd_head_bwd", _lib.ptr(x), _lib.ptr(w), _lib.ptr(dpad), _lib.ptr(pmy), _lib.ptr(dl), _lib.ptr(dx),
                  _lib.ptr(dwide), _lib.ptr(part), _lib.ptr(grads), B, H, Dp, _lib.stream())
        return (dx, grads[:H].view(wshape).to(wdt), grads[H + Dp:].view(bshape).to(bdt), dwide, None,
                grads[H:H + Dp].view(wdshape).to(wddt), None)


def head_fusable(x: torch.Tensor, dpad: torch.Tensor) -> bool:
    return (FUSED_HEAD and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.is_contiguous()
            and x.shape[1] % 8 == 0 and x.shape[1] <= 512 and dpad.shape[1] <= 64 and x.data_ptr() % 16 == 0)


FUSED_HEAD = os.environ.get("KFA_WD_FUSED_HEAD", "1") != "0"  # csrc/kernels/widedeep.hip
FUSED_INPUT = os.environ.get("KFA_WD_FUSED_INPUT", "1") != "0"  # csrc/kernels/widedeep.hip
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

    def forward(self, dense: torch.Tensor, ids: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        B, nf = ids.shape
        gids = (ids + self.offsets.view(1, nf)).reshape(-1)
        flat_rows = self.tables(gids, getattr(ids, "_kfa_plan", None))  # [B*nf, E+8]
        cdt = self.weights[0].dtype
        dpad = F.pad(dense, (0, cfg.dense_pad - cfg.num_dense))
        if (FUSED_INPUT and flat_rows.is_cuda and flat_rows.dtype == torch.bfloat16 and cdt == torch.bfloat16
                and cfg.embed_dim % 8 == 0 and flat_rows.is_contiguous()):
            x, wide = _WDInputFn.apply(flat_rows, dpad.float().contiguous(), B, nf, cfg.embed_dim)
        else:
            rows = flat_rows.view(B, nf, cfg.row_width)  # [B, nf, E+8]
            deep_emb = rows[:, :, :cfg.embed_dim].reshape(B, nf * cfg.embed_dim)
            wide = rows[:, :, cfg.embed_dim].float().sum(1)
            x = torch.cat([dpad.to(rows.dtype), deep_emb], 1)
        if x.is_cuda:
            x = x.to(cdt)
            for w, b in zip(self.weights, self.biases):
                x = T.dense(x, w, b, "relu")
        else:
            x = x.float()
            for w, b in zip(self.weights, self.biases):
                x = torch.relu(x @ w.float().t() + b.float())
        dpad32 = dpad.float().contiguous()
        if head_fusable(x, dpad32):
            return _WDHeadFn.apply(x, self.out_w, self.out_b, wide, dpad32, self.wide_dense, labels)
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
