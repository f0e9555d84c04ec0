"""BERT pre-training (MLM + NSP) — BASELINE.json config "BERT-base pretrain,
4 workers + 2 PS, RCCL push/pull grad sync" (SURVEY §2.6 K1/K2/K4/K6/K10/K11).

MI355X path (``x.is_cuda``): every encoder layer is one
:class:`~kubeflow_controller_amd.ops.transformer.EncoderLayerFn` node
(hipBLASLt GEMMs + fused HIP epilogue / LayerNorm / softmax / layout kernels,
explicit backward with direct flat-buffer gradients), the embedding lookup and
its sparse backward are HIP kernels, and the MLM decoder (tied to the word
embedding) is fused with the softmax-cross-entropy kernel (decoder bias added
inside the loss kernel; dlogits produced in the forward pass).

CPU path: the same parameters through plain PyTorch fp32 ops (no dropout) —
used by CPU replicas and as the numerics reference of the GPU path.

Vocabulary is padded to a multiple of 64 (30522 → 30528) so the decoder GEMM
and the loss kernel run on aligned rows; padded ids never occur as inputs or
labels.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import transformer as T
from ..ops.loss import classifier_xent


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    hidden_dropout: float = 0.1
    attn_dropout: float = 0.1
    ln_eps: float = 1e-12
    init_range: float = 0.02
    max_predictions: int = 20   # masked positions per sequence (S=128 recipe)

    @classmethod
    def base(cls) -> "BertConfig":
        return cls()

    @classmethod
    def large(cls) -> "BertConfig":
        return cls(hidden=1024, layers=24, heads=16, intermediate=4096)

    @classmethod
    def tiny(cls) -> "BertConfig":
        return cls(vocab_size=1000, hidden=128, layers=2, heads=2, intermediate=512, max_position=128,
                   max_predictions=8)

    @property
    def padded_vocab(self) -> int:
        return (self.vocab_size + 63) // 64 * 64


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig):
        super().__init__()
        H, I = cfg.hidden, cfg.intermediate
        self.wqkv = nn.Parameter(torch.empty(3 * H, H))
        self.bqkv = nn.Parameter(torch.zeros(3 * H))
        self.wo = nn.Parameter(torch.empty(H, H))
        self.bo = nn.Parameter(torch.zeros(H))
        self.ln1_g = nn.Parameter(torch.ones(H))
        self.ln1_b = nn.Parameter(torch.zeros(H))
        self.w1 = nn.Parameter(torch.empty(I, H))
        self.b1 = nn.Parameter(torch.zeros(I))
        self.w2 = nn.Parameter(torch.empty(H, I))
        self.b2 = nn.Parameter(torch.zeros(H))
        self.ln2_g = nn.Parameter(torch.ones(H))
        self.ln2_b = nn.Parameter(torch.zeros(H))
        for w in (self.wqkv, self.wo, self.w1, self.w2):
            nn.init.normal_(w, 0.0, cfg.init_range)

    def params(self):
        return (self.wqkv, self.bqkv, self.wo, self.bo, self.ln1_g, self.ln1_b, self.w1, self.b1, self.w2, self.b2,
                self.ln2_g, self.ln2_b)


class BertForPreTraining(nn.Module):
    def __init__(self, cfg: BertConfig, seed: int = 0):
        super().__init__()
        self.cfg = cfg
        H, V = cfg.hidden, cfg.padded_vocab
        self.word_emb = nn.Parameter(torch.empty(V, H))
        self.pos_emb = nn.Parameter(torch.empty(cfg.max_position, H))
        self.type_emb = nn.Parameter(torch.empty(cfg.type_vocab, H))
        for w in (self.word_emb, self.pos_emb, self.type_emb):
            nn.init.normal_(w, 0.0, cfg.init_range)
        self.emb_ln_g = nn.Parameter(torch.ones(H))
        self.emb_ln_b = nn.Parameter(torch.zeros(H))
        self.layers = nn.ModuleList(BertLayer(cfg) for _ in range(cfg.layers))
        # MLM head: transform (dense + GELU + LN), decoder tied to word_emb (+ bias)
        self.mlm_w = nn.Parameter(torch.empty(H, H))
        self.mlm_b = nn.Parameter(torch.zeros(H))
        self.mlm_ln_g = nn.Parameter(torch.ones(H))
        self.mlm_ln_b = nn.Parameter(torch.zeros(H))
        self.dec_b = nn.Parameter(torch.zeros(V))
        # NSP head: pooler (dense + tanh on [CLS]) + 2-way classifier
        self.pool_w = nn.Parameter(torch.empty(H, H))
        self.pool_b = nn.Parameter(torch.zeros(H))
        self.nsp_w = nn.Parameter(torch.empty(2, H))
        self.nsp_b = nn.Parameter(torch.zeros(2))
        for w in (self.mlm_w, self.pool_w, self.nsp_w):
            nn.init.normal_(w, 0.0, cfg.init_range)
        # the word embedding is written by two direct-gradient kernels per step; the
        # module-level map survives copy.deepcopy (a Parameter's own attributes do
        # not), the Engine re-applies it (trainer/engine.py)
        self.word_emb._kfa_uses = 2
        self._kfa_param_uses = {"word_emb": 2}
        self.seed = seed
        self._step = 0
        self._pos_cache = {}

    @property
    def graph_capturable(self) -> bool:
        """Dropout masks come from per-step host seeds: a replayed HIP graph would
        repeat one step's masks (``Engine.graph_ok``)."""
        return not (self.training and (self.cfg.hidden_dropout > 0 or self.cfg.attn_dropout > 0))

    # ------------------------------------------------------------------ helpers
    def _pos_ids(self, B, S, device):
        key = (B, S, str(device))
        t = self._pos_cache.get(key)
        if t is None:
            t = torch.arange(S, device=device).repeat(B)
            self._pos_cache[key] = t
        return t

    def _cls_rows(self, B, S, device):
        key = ("cls", B, S, str(device))
        t = self._pos_cache.get(key)
        if t is None:
            t = torch.arange(B, device=device, dtype=torch.int64) * S
            self._pos_cache[key] = t
        return t

    @staticmethod
    def key_bias(attention_mask):
        if attention_mask is None:
            return None
        return ((1.0 - attention_mask.float()) * -10000.0).contiguous()

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids, token_type_ids, attention_mask, mlm_positions, mlm_labels, nsp_labels):
        if not input_ids.is_cuda:
            return self.forward_reference(input_ids, token_type_ids, attention_mask, mlm_positions, mlm_labels,
                                          nsp_labels)
        cfg = self.cfg
        B, S = input_ids.shape
        H = cfg.hidden
        dev = input_ids.device
        ph = cfg.hidden_dropout if self.training else 0.0
        pa = cfg.attn_dropout if self.training else 0.0
        step_seed = T.mix_seed(self.seed, self._step)
        if self.training:
            self._step += 1
        e = T.embedding_sum([self.word_emb, self.pos_emb, self.type_emb],
                            [input_ids.reshape(-1), self._pos_ids(B, S, dev), token_type_ids.reshape(-1)])
        h = T.layer_norm(e, self.emb_ln_g, self.emb_ln_b, cfg.ln_eps)
        if ph > 0:
            h = T.dense_dropout(h, ph, T.mix_seed(step_seed, 999))
        kb = self.key_bias(attention_mask)
        # layer i+1's QKV-projection dgrad reaches layer i's LN2 backward through a
        # ResidualJoin (summed on read) instead of a GEMM addend (ops/transformer.py)
        join_in = None
        for i, layer in enumerate(self.layers):
            join_out = T.ResidualJoin() if (self.training and i + 1 < len(self.layers)) else None
            lcfg = (B, S, cfg.heads, ph, pa, T.s64(T.mix_seed(step_seed, i)), cfg.ln_eps, join_in, join_out)
            h = T.EncoderLayerFn.apply(h, kb, lcfg, *layer.params())
            join_in = join_out
        # the masked positions (MLM) and the [CLS] rows (NSP) in ONE gather: its backward
        # is one zero-fill + one index_add into [T, H] instead of two and a sum of them
        pos = mlm_positions.reshape(-1)
        rows = torch.cat([pos.to(torch.int64), self._cls_rows(B, S, dev)])
        g = h.index_select(0, rows)
        hm, hc = g[:pos.numel()], g[pos.numel():]
        t = T.dense(hm, self.mlm_w, self.mlm_b, "gelu")
        t = T.layer_norm(t, self.mlm_ln_g, self.mlm_ln_b, cfg.ln_eps)
        mlm = T.decoder_xent(t, self.word_emb, self.dec_b, mlm_labels.reshape(-1))
        # NSP on [CLS]
        pooled = T.dense(hc, self.pool_w, self.pool_b, "tanh")
        nsp = classifier_xent(pooled.contiguous(), self.nsp_w, self.nsp_b, nsp_labels)  # fused 2-way head + loss
        return mlm + nsp

    def forward_reference(self, input_ids, token_type_ids, attention_mask, mlm_positions, mlm_labels, nsp_labels):
        """Plain PyTorch fp32, no dropout (CPU replicas + numerics reference)."""
        cfg = self.cfg
        B, S = input_ids.shape
        H = cfg.hidden
        f = lambda t: t.float()  # noqa: E731
        pos = torch.arange(S, device=input_ids.device)
        e = f(self.word_emb)[input_ids] + f(self.pos_emb)[pos][None] + f(self.type_emb)[token_type_ids]
        h = F.layer_norm(e, (H,), f(self.emb_ln_g), f(self.emb_ln_b), cfg.ln_eps).reshape(B * S, H)
        kb = self.key_bias(attention_mask)
        for layer in self.layers:
            h = T.encoder_layer_reference(h, kb, (B, S, cfg.heads, 0.0, 0.0, 0, cfg.ln_eps), *layer.params())
        hm = h.index_select(0, mlm_positions.reshape(-1))
        t = F.gelu(hm @ f(self.mlm_w).t() + f(self.mlm_b))
        t = F.layer_norm(t, (H,), f(self.mlm_ln_g), f(self.mlm_ln_b), cfg.ln_eps)
        logits = t @ f(self.word_emb).t() + f(self.dec_b)
        mlm = F.cross_entropy(logits, mlm_labels.reshape(-1))
        pooled = torch.tanh(h.view(B, S, H)[:, 0] @ f(self.pool_w).t() + f(self.pool_b))
        nsp = F.cross_entropy(pooled @ f(self.nsp_w).t() + f(self.nsp_b), nsp_labels)
        return mlm + nsp


def bert_loss(model, *batch):
    return model(*batch)


def synthetic_mlm_batch(cfg: BertConfig, batch: int, seq_len: int, generator=None, device="cpu"):
    """Random token ids / segment split / masked positions of the pre-training
    shapes (no network: no corpus). Returns the positional args of forward()."""
    g = generator
    B, S = batch, seq_len
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
    split = torch.randint(S // 4, 3 * S // 4, (B, 1), generator=g)
    tt = (torch.arange(S)[None, :] >= split).long()
    n = min(cfg.max_predictions, S)
    pos = torch.stack([torch.randperm(S, generator=g)[:n] for _ in range(B)]).sort(1).values
    flat = (pos + torch.arange(B)[:, None] * S).reshape(-1)
    labels = torch.randint(0, cfg.vocab_size, (B * n,), generator=g)
    nsp = torch.randint(0, 2, (B,), generator=g)
    to = lambda t: t.to(device)  # noqa: E731
    return to(ids), to(tt), None, to(flat), to(labels), to(nsp)


def flops_per_step(cfg: BertConfig, batch: int, seq_len: int) -> float:
    """Model FLOPs (fwd+bwd = 3x fwd) of one pre-training step."""
    Tk = batch * seq_len
    H, I, L = cfg.hidden, cfg.intermediate, cfg.layers
    per_layer = 2 * Tk * (3 * H * H + H * H + 2 * H * I) + 2 * 2 * batch * seq_len * seq_len * H
    n_pred = batch * min(cfg.max_predictions, seq_len)
    head = 2 * n_pred * (H * H + H * cfg.padded_vocab)
    return 3.0 * (L * per_layer + head)
