"""BERT FFN-up forward (32768 x 3072 x 768, bias + GELU): hipBLASLt + the bias/GELU pass,
the own wave-specialised GEMM + pass, the persistent GEMM with the GELU epilogue (ppp),
and the wave-specialised GEMM with the GELU store epilogue (ppw, plain / non-temporal
stores).  Correctness vs fp32 first; CUDA-event timing, interleaved, min of medians."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops.transformer import bias_act_fwd  # noqa: E402


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
    M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (32768, 3072, 768)))
    torch.manual_seed(0)
    h = torch.randn(M, K, device=d).to(torch.bfloat16)
    w = (torch.randn(N, K, device=d) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=d) * 0.1
    zr = h.float() @ w.float().t() + b
    yr = torch.nn.functional.gelu(zr)
    ppw_gelu = getattr(G, "gemm_ppw_gelu", None)  # the reverted round-6 experiment (docs/kernels.md)
    for nt in ((False, True) if ppw_gelu else ()):
        y, z = ppw_gelu(h, w, b, nt=nt)
        print(f"ppw-gelu nt={nt}: max|z-zr| {(z.float() - zr).abs().max().item():.4f} "
              f"max|y-yr| {(y.float() - yr).abs().max().item():.4f}", flush=True)
    cands = {
        "hipblaslt+pass": lambda: bias_act_fwd(torch.mm(h, w.t()), b, "gelu"),
        "ppw256-nt+pass": lambda: bias_act_fwd(G.gemm_ppp(h, w, probe=10, split=False), b, "gelu"),
        "ppp256-gelu": lambda: G.gemm_ppp_gelu(h, w, b),
        "hipblaslt (bare)": lambda: torch.mm(h, w.t()),
    }
    if ppw_gelu:
        cands["ppw256-gelu"] = lambda: ppw_gelu(h, w, b)
        cands["ppw256-nt-gelu"] = lambda: ppw_gelu(h, w, b, nt=True)
    res = {k: [] for k in cands}
    for _ in range(2):
        for k, f in cands.items():
            res[k].append(t(f))
    for k, v in res.items():
        print(f"{M}x{N}x{K} {k:18s} {min(v):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
