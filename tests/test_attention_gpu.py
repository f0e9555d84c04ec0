"""Fused attention (csrc/kernels/attention.hip) vs a plain PyTorch fp32 reference.

The dropout case rebuilds the kernels' counter-hash keep mask in numpy (numpy copy
of drop_hash in csrc/kernels/common.h, one hash per (q, k) / (q, k + 16) score pair,
16-bit halves against round(p·2^16) — attention.hip attn_pair_hash) so forward AND
backward are checked element-wise against the reference with the identical mask;
the S = 128 backward runs both from the forward's packed mask and re-hashing."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

D = torch.device("cuda")


def _close(a, b, tol, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert err <= tol * scale, f"{what}: err {err} scale {scale}"


def _drop_hash(seed, i):
    """numpy copy of drop_hash (csrc/kernels/common.h) over uint64 indices."""
    s = np.uint64(seed)
    k0 = np.uint32(int(s) & 0xFFFFFFFF)
    k1 = np.uint32(int(s) >> 32)
    with np.errstate(over="ignore"):
        lo = (i & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (i >> np.uint64(32)).astype(np.uint32)
        x = (lo ^ k0) + k1 + (hi & np.uint32(0xFFFFFF)) * np.uint32(0x9E3779)
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def _t16(p):
    return min(int(p * 65536.0 + 0.5), 65536)


def _keep_mask(seed, B, heads, S, p):
    """[B, heads, S, S] keep mask: pair (row, k) / (row, k + 16) (k with bit 4 clear)
    shares the hash of index row·S + k; low half decides k, high half k + 16."""
    from kubeflow_controller_amd.ops.transformer import hash_key  # the launch key the wrapper passes
    key = np.arange(S, dtype=np.uint64)
    rows = np.arange(B * heads * S, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(S) + (key & ~np.uint64(16))[None, :]
    h = _drop_hash(hash_key(seed), idx)
    half = np.where((key & np.uint64(16)) != 0, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return torch.from_numpy((half >= _t16(p)).reshape(B, heads, S, S).astype(np.float32))


def _reference(qkv, bqkv, kb, B, S, heads, d, mask, p):
    x = qkv + bqkv
    q, k, v = x.view(B, S, 3, heads, d).permute(2, 0, 3, 1, 4)
    sc = q @ k.transpose(-1, -2) / math.sqrt(d)
    if kb is not None:
        sc = sc + kb.view(B, 1, 1, S)
    pr = torch.softmax(sc, -1)
    if mask is not None:
        pr = pr * mask / (1.0 - _t16(p) / 65536.0)
    return (pr @ v).permute(0, 2, 1, 3).reshape(B * S, heads * d)


@pytest.mark.parametrize("S", [128, 256, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_attention_fwd_bwd(p, S):
    """S = 128: one workgroup per head; S = 256 / 512: the 128-block kernels
    (online-softmax forward, key-owner dK/dV + query-owner dQ backward)."""
    from kubeflow_controller_amd.ops import transformer as T
    torch.manual_seed(0)
    B, heads, d = (3, 4, 64) if S == 128 else (2, 2, 64)
    H = heads * d
    qkv = torch.randn(B * S, 3 * H, device=D).to(torch.bfloat16)
    bqkv = torch.randn(3 * H, device=D) * 0.1
    m = torch.ones(B, S, device=D)
    m[1, S - 38:] = 0   # masked tail, crossing a 128-key block boundary for S > 128
    kb = ((1 - m) * -10000.0).contiguous()
    seed = 987654321
    out, lse, kmask = T.attn_fwd(qkv, bqkv, kb, B, S, heads, p, seed, want_mask=True)
    assert (kmask is not None) == (p > 0 and S == 128)
    mask = _keep_mask(seed, B, heads, S, p).to(D) if p > 0 else None
    xr = qkv.float().requires_grad_()
    br = bqkv.clone().requires_grad_()
    ref = _reference(xr, br, kb, B, S, heads, d, mask, p)
    _close(out, ref, 2e-2, "ctx")
    dout = torch.randn(B * S, H, device=D)
    ref.backward(dout)
    db = torch.zeros(3 * H, device=D)
    dqkv = T.attn_bwd(qkv, bqkv, kb, out, lse, dout.to(torch.bfloat16), db, B, S, heads, p, seed, mask=kmask)
    _close(dqkv, xr.grad, 3e-2, "dqkv")
    _close(db, br.grad, 3e-2, "dbqkv")
    if kmask is not None:  # the re-hashing backward: the same decisions, bit for bit the same result
        dqkv_h = T.attn_bwd(qkv, bqkv, kb, out, lse, dout.to(torch.bfloat16), None, B, S, heads, p, seed)
        assert torch.equal(dqkv_h, dqkv)
        # the packed words: word [bh][c][q] bit (k >> 4)·4 + (k & 3) for the keys with (k >> 2) & 3 == c
        m = mask.view(B * heads, S, S).to(torch.int64).cpu()
        k = torch.arange(S)
        bit = (k >> 4) * 4 + (k & 3)
        words = torch.zeros(B * heads, 4, S, dtype=torch.int64)
        for c in range(4):
            sel = ((k >> 2) & 3) == c
            words[:, c, :] = (m[:, :, sel] << bit[sel]).sum(-1)
        assert torch.equal(kmask.cpu().to(torch.int64) & 0xFFFFFFFF, words)


def test_fused_attention_lse_matches():
    from kubeflow_controller_amd.ops import transformer as T
    torch.manual_seed(1)
    B, S, heads, d = 2, 128, 2, 64
    H = heads * d
    qkv = torch.randn(B * S, 3 * H, device=D).to(torch.bfloat16)
    bqkv = torch.zeros(3 * H, device=D)
    _, lse = T.attn_fwd(qkv, bqkv, None, B, S, heads)
    q, k, _ = qkv.float().view(B, S, 3, heads, d).permute(2, 0, 3, 1, 4)
    ref = torch.logsumexp((q @ k.transpose(-1, -2)) / math.sqrt(d), -1)   # [B, heads, S]
    _close(lse.view(B, heads, S), ref, 2e-2, "lse")
