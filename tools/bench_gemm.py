"""GEMM / attention microbenchmark on MI355X.

Dense: hipBLASLt (``torch.mm``) vs the hand-written MFMA GEMM
(``ops/gemm.py``, both tile widths) for Y = X·Wᵀ, and hipBLASLt vs the
hand-written wgrad kernel for dW = dYᵀ·X, on the BERT-base / Wide&Deep shapes.
Attention (BERT-base, S = 128, d = 64): the fused kernel each way vs the split
path (QKV split, batched library GEMMs, softmax kernel).  Prints ms and TFLOP/s.
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops import transformer as T  # noqa: E402
from kubeflow_controller_amd.ops.conv import wgrad_into  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def dense():
    d = torch.device("cuda")
    shapes = [(32768, 2304, 768), (32768, 768, 768), (32768, 3072, 768), (32768, 768, 3072),
              (8192, 2304, 768), (8192, 768, 3072), (65536, 1024, 1680), (65536, 512, 1024), (8192, 8192, 8192)]
    print(f"{'M':>6} {'N':>5} {'K':>5} | {'mm ms':>7} {'TF/s':>5} | {'g128':>7} {'TF/s':>5} | {'g256':>7} {'TF/s':>5}"
          f" | {'gelu+z':>7} | {'wg mm':>7} {'TF/s':>5} | {'wg kfa':>7} {'TF/s':>5}")
    for M, N, K in shapes:
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, device=d).to(torch.bfloat16)
        b = torch.randn(N, device=d)
        dy = torch.randn(M, N, device=d).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        t_mm = timeit(lambda: torch.mm(x, w.t()))
        t_128 = timeit(lambda: G.gemm_nt(x, w, bn=128))
        t_256 = timeit(lambda: G.gemm_nt(x, w, bn=256))
        t_128o = timeit(lambda: G.gemm_nt(x, w, bn=128, persistent=1))
        t_256o = timeit(lambda: G.gemm_nt(x, w, bn=256, persistent=1))
        t_2cu = timeit(lambda: G.gemm_nt(x, w, persistent=3))
        t_2cu4 = timeit(lambda: G.gemm_nt(x, w, persistent=4))
        t_pp = timeit(lambda: G.gemm_nt(x, w, persistent=5))
        t_ppp = timeit(lambda: G.gemm_nt(x, w, persistent=6))
        t_noepi = timeit(lambda: G.gemm_nt(x, w, persistent=7))
        t_pppe = timeit(lambda: G.gemm_nt(x, w, bias=b, act="gelu", want_z=True, persistent=6))
        t_ep = timeit(lambda: G.gemm_nt(x, w, bias=b, act="gelu", want_z=True))
        gw = torch.zeros(N, K, device=d, dtype=torch.bfloat16)
        t_wm = timeit(lambda: gw.addmm_(dy.t(), x))
        t_wk = timeit(lambda: wgrad_into(x, dy, gw, 1, 1, M, K, 1, M, N, 1, 1, 1, 0, True))
        tf = lambda t: fl / t / 1e9  # noqa: E731
        print(f"{M:6d} {N:5d} {K:5d} | {t_mm:7.3f} {tf(t_mm):5.0f} | {t_128:7.3f} {tf(t_128):5.0f} | "
              f"{t_256:7.3f} {tf(t_256):5.0f} | {t_ep:7.3f} | {t_wm:7.3f} {tf(t_wm):5.0f} | {t_wk:7.3f} {tf(t_wk):5.0f}"
              f" | persistent: g128 {tf(t_128o):5.0f} g256 {tf(t_256o):5.0f} | 2/CU g128 {tf(t_2cu):5.0f} 4w {tf(t_2cu4):5.0f} | pingpong {tf(t_pp):5.0f} nt-stores {tf(t_ppp):5.0f} (+bias/gelu/z {t_pppe:.3f} ms) | pp main loop only {tf(t_noepi):5.0f} TF/s",
              flush=True)


def attention():
    d = torch.device("cuda")
    B, S, heads, hd = 256, 128, 12, 64
    H = heads * hd
    qkv = torch.randn(B * S, 3 * H, device=d).to(torch.bfloat16)
    bqkv = torch.randn(3 * H, device=d) * 0.1
    kb = torch.zeros(B, S, device=d)
    dout = torch.randn(B * S, H, device=d).to(torch.bfloat16)
    fl = 4.0 * B * heads * S * S * hd
    for p in (0.0, 0.1):
        t_f = timeit(lambda: T.attn_fwd(qkv, bqkv, kb, B, S, heads, p, 1))
        out, lse = T.attn_fwd(qkv, bqkv, kb, B, S, heads, p, 1)
        db = torch.zeros(3 * H, device=d)
        t_b = timeit(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, heads, p, 1))

        def split_fwd():
            x = (qkv.float() + bqkv).to(torch.bfloat16).view(B, S, 3, heads, hd).permute(2, 0, 3, 1, 4)
            q, k, v = x[0], x[1], x[2]
            sc = torch.matmul(q, k.transpose(-1, -2)) * (1.0 / math.sqrt(hd)) + kb.view(B, 1, 1, S).to(q.dtype)
            pr = torch.softmax(sc.float(), -1).to(q.dtype)
            if p > 0:
                pr = torch.nn.functional.dropout(pr, p)
            return torch.matmul(pr, v)
        t_s = timeit(split_fwd)
        print(f"attention B={B} S={S} heads={heads} p={p}: fused fwd {t_f:.3f} ms ({fl / t_f / 1e9:.0f} TF/s), "
              f"fused bwd {t_b:.3f} ms ({2.5 * fl / t_b / 1e9:.0f} TF/s), torch split fwd {t_s:.3f} ms", flush=True)


def wgrad_layouts():
    """hipBLASLt on the weight-gradient contraction over tokens, every operand layout."""
    d = torch.device("cuda")
    for M, N, K in [(32768, 2304, 768), (32768, 768, 768), (32768, 3072, 768), (32768, 768, 3072)]:
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        dy = torch.randn(M, N, device=d).to(torch.bfloat16)
        xt, dyt = x.t().contiguous(), dy.t().contiguous()
        fl = 2.0 * M * N * K
        r = {
            "dy.t()@x": timeit(lambda: torch.mm(dy.t(), x)),
            "x.t()@dy": timeit(lambda: torch.mm(x.t(), dy)),
            "dyT@xT.t()": timeit(lambda: torch.mm(dyt, xt.t())),
            "dyT@x": timeit(lambda: torch.mm(dyt, x)),
            "transpose dy": timeit(lambda: dy.t().contiguous()),
        }
        print(f"wgrad {M}x{N}x{K}: " + ", ".join(f"{k} {v:.3f} ms ({fl / v / 1e9:.0f} TF/s)" for k, v in r.items()),
              flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["dense", "attention", "wgrad_layouts"]
    for w in what:
        globals()[w]()
