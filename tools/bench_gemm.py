"""GEMM microbenchmark on MI355X: hipBLASLt (torch.mm) vs the hand-written MFMA
kernels (conv_igemm as a 1x1 conv for Y = X·Wᵀ; wgrad for dW = dYᵀ·X) on the
BERT-base / Wide&Deep / ResNet shapes.  Prints TFLOP/s per shape."""
import sys
import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
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


def main():
    d = torch.device("cuda")
    shapes = [(8192, 2304, 768), (8192, 768, 768), (8192, 3072, 768), (8192, 768, 3072),
              (16384, 3072, 768), (16384, 768, 3072), (8192, 1024, 1680), (802816, 256, 64), (200704, 512, 128)]
    print(f"{'M':>7} {'N':>5} {'K':>5} | {'mm ms':>7} {'TF/s':>6} | {'igemm':>7} {'TF/s':>6} | "
          f"{'wg mm':>7} {'TF/s':>6} | {'wg kfa':>7} {'TF/s':>6}")
    for M, N, K in shapes:
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, device=d).to(torch.bfloat16)
        dy = torch.randn(M, N, device=d).to(torch.bfloat16)
        y = torch.empty(M, N, device=d, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t_mm = timeit(lambda: torch.mm(x, w.t()))
        variant = 1 if N <= 64 else 0

        def ig():
            _lib.call("kfa_conv_igemm", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, 1, 1, M, K, 1, M, 1, 1, 1, 1,
                      0, 0, N, 1, M, 1, 0, 0, N, variant, _lib.stream())
        t_ig = timeit(ig) if K % 64 == 0 else float("nan")
        gw = torch.zeros(N, K, device=d, dtype=torch.bfloat16)
        t_wm = timeit(lambda: gw.addmm_(dy.t(), x))
        t_wk = timeit(lambda: wgrad_into(x, dy, gw, 1, 1, M, K, 1, M, N, 1, 1, 1, 0, True))
        print(f"{M:7d} {N:5d} {K:5d} | {t_mm:7.3f} {fl / t_mm / 1e9:6.0f} | {t_ig:7.3f} {fl / t_ig / 1e9:6.0f} | "
              f"{t_wm:7.3f} {fl / t_wm / 1e9:6.0f} | {t_wk:7.3f} {fl / t_wk / 1e9:6.0f}", flush=True)
    # numerics spot check of the igemm-as-GEMM path
    M, N, K = 4096, 768, 768
    x = torch.randn(M, K, device=d).to(torch.bfloat16)
    w = torch.randn(N, K, device=d).to(torch.bfloat16)
    y = torch.empty(M, N, device=d, dtype=torch.bfloat16)
    _lib.call("kfa_conv_igemm", _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, 1, 1, M, K, 1, M, 1, 1, 1, 1,
              0, 0, N, 1, M, 1, 0, 0, N, 0, _lib.stream())
    ref = x.float() @ w.float().t()
    print("igemm-as-GEMM max rel err", ((y.float() - ref).abs().max() / ref.abs().max()).item())


if __name__ == "__main__":
    main()
