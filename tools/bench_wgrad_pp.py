"""Pointwise weight gradients (dense dW = dYᵀ·X, 1x1 convs) on the current wgrad
route: run once with KFA_WGRAD_PP=1 (ping-pong wgrad_pp_kernel) and once with 0
(lockstep wgrad_kernel<2,4,8,4>).  Prints ms and TFLOP/s per shape (incl. the
split-K reduce)."""
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.conv import wgrad_into  # noqa: E402

SHAPES = [(32768, 2304, 768), (32768, 768, 768), (32768, 3072, 768), (32768, 768, 3072), (65536, 1024, 1680),
          # ResNet-50 bs 256 pointwise convs (pixels, Cout, Cin)
          (802816, 256, 64), (802816, 64, 256), (802816, 128, 256), (200704, 512, 128), (200704, 128, 512),
          (200704, 256, 512), (50176, 1024, 256), (50176, 256, 1024), (50176, 512, 1024), (12544, 2048, 512),
          (12544, 512, 2048), (200704, 512, 256), (50176, 1024, 512), (12544, 2048, 1024)]
d = torch.device("cuda")
for rows, co, ci in SHAPES:
    x = torch.randn(rows, ci, device=d).to(torch.bfloat16)
    dy = torch.randn(rows, co, device=d).to(torch.bfloat16)
    out = torch.zeros(co, ci, device=d)
    f = lambda: wgrad_into(x, dy, out, 1, 1, rows, ci, 1, rows, co, 1, 1, 1, 0, accumulate=True)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 10)
    print(f"PP={os.environ.get('KFA_WGRAD_PP', '1')} {rows}x{co}x{ci}: {best * 1e3:8.1f} us "
          f"{2 * rows * co * ci / best / 1e9:6.0f} TF/s", flush=True)
