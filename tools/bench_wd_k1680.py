"""W&D first MLP layer (65536 x 1024 x K=1680): is the forward slow because the rows of
x (1680 bf16 = 3360 B) and of W1 are not 128-B aligned?  Times the own bias+ReLU GEMM and
hipBLASLt on (a) contiguous K = 1680 operands, (b) the same K with 128-B aligned row
strides (views into [*, 1728] buffers), (c) zero-padded K = 1728.  CUDA-event timing,
interleaved rounds, min of medians."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(out)


def main():
    d = torch.device("cuda")
    M, N, K, KP = 65536, 1024, 1680, 1728
    torch.manual_seed(0)
    xp = torch.zeros(M, KP, device=d, dtype=torch.bfloat16)
    wp = torch.zeros(N, KP, device=d, dtype=torch.bfloat16)
    xp[:, :K] = torch.randn(M, K, device=d).to(torch.bfloat16)
    wp[:, :K] = (torch.randn(N, K, device=d) * K ** -0.5).to(torch.bfloat16)
    x = xp[:, :K].contiguous()
    w = wp[:, :K].contiguous()
    xs, ws = xp[:, :K], wp[:, :K]          # strided views: rows 3456 B apart
    bias = torch.randn(N, device=d)
    ref = torch.relu(x.float() @ w.float().t() + bias)
    for name, a, b in (("contig", x, w), ("strided", xs, ws), ("strided-x", xs, w), ("padK", xp, wp)):
        y = G.gemm_ppp_relu(a, b, bias)
        err = (y.float() - ref).abs().max().item()
        r = []
        for _ in range(2):
            r.append((t(lambda: G.gemm_ppp_relu(a, b, bias)), t(lambda: torch.mm(a, b.t()))))
        own = min(v[0] for v in r)
        lib = min(v[1] for v in r)
        print(f"{name:10s} lda={a.stride(0)} ldb={b.stride(0)} K={a.shape[1]}: ppp256-relu {own:7.1f} us  "
              f"hipBLASLt {lib:7.1f} us  max|err| {err:.3f}", flush=True)




def gm_sweep():
    """KFA_GM_SWEEP=1: the persistent kernels' tile-raster group height (256-row tiles
    per group; 4 = default) on the layer's forward and data-gradient shapes and on the
    BERT FFN-up shape."""
    from kubeflow_controller_amd.ops import _lib
    _lib.register("kfa_gemm_ppp_set_gm", [_lib.I])
    L = _lib.lib()
    d = torch.device("cuda")
    for M, N, K in ((65536, 1024, 1680), (65536, 1680, 1024), (32768, 3072, 768), (65536, 512, 1024)):
        a = torch.randn(M, K, device=d).to(torch.bfloat16)
        b = (torch.randn(N, K, device=d) * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=d)
        out = []
        for gm in (1, 2, 4, 8, 16, 32):
            L.kfa_gemm_ppp_set_gm(gm)
            out.append(f"gm{gm}: relu {t(lambda: G.gemm_ppp_relu(a, b, bias)):6.1f} ppw {t(lambda: G.gemm_ppp(a, b, probe=9, split=False)):6.1f}")
        L.kfa_gemm_ppp_set_gm(0)
        print(f"{M}x{N}x{K} hipBLASLt {t(lambda: torch.mm(a, b.t())):6.1f} | " + " | ".join(out), flush=True)


def pmc_mode():
    """Short fixed-order run for a rocprofv3 --pmc pass: own fwd (K = 1680), own on the
    layer's data-gradient shape (65536 x 1680 x 1024, same FLOPs), hipBLASLt fwd."""
    d = torch.device("cuda")
    M, N, K = 65536, 1024, 1680
    x = torch.randn(M, K, device=d).to(torch.bfloat16)
    w = (torch.randn(N, K, device=d) * K ** -0.5).to(torch.bfloat16)
    dz = torch.randn(M, N, device=d).to(torch.bfloat16)
    wt = w.t().contiguous()
    bias = torch.randn(N, device=d)
    for _ in range(6):
        G.gemm_ppp_relu(x, w, bias)
    for _ in range(6):
        G.gemm_ppp(dz, wt, probe=9, split=False)
    for _ in range(6):
        torch.mm(x, w.t())
    torch.cuda.synchronize()


if __name__ == "__main__":
    if os.environ.get("KFA_PMC_MODE") == "1":
        pmc_mode()
    elif os.environ.get("KFA_GM_SWEEP") == "1":
        gm_sweep()
    else:
        main()
