"""gemm_ppw_kernel (probe 9 / 10: plain / non-temporal C stores) on the BERT-base
and W&D dense shapes: median of 5 x 30 launches per shape, random bf16 operands.
Run once per kernel library (KFA_KERNELS_SO) for a same-box A/B."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.gemm import gemm_ppp  # noqa: E402

SHAPES = [(32768, 2304, 768), (32768, 768, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 2304),
          (65536, 1024, 1680)]
d = torch.device("cuda")
for m, n, k in SHAPES:
    a = torch.randn(m, k, device=d).to(torch.bfloat16)
    b = torch.randn(n, k, device=d).to(torch.bfloat16)
    for probe in (9, 10):
        f = lambda: gemm_ppp(a, b, probe=probe, split=False)  # noqa: E731
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(30):
                f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 30)
        t = statistics.median(ts)
        print(f"ppw{'-nt' if probe == 10 else '   '} {m}x{n}x{k}: {t * 1e3:8.1f} us {2 * m * n * k / t / 1e9:6.0f} TF/s", flush=True)
