"""Weight-gradient GEMM layouts on hipBLASLt vs the hand-written wgrad kernel (BERT shapes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.conv import wgrad_into  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


d = torch.device("cuda")
for (M, N, K) in [(16384, 3072, 768), (16384, 2304, 768), (16384, 768, 3072), (16384, 768, 768), (8192, 2304, 768)]:
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=d, dtype=torch.bfloat16)
    gwt = torch.zeros(K, N, device=d, dtype=torch.bfloat16)
    fl = 2 * M * N * K
    res = {
        "addmm_(dyT,x)": t(lambda: gw.addmm_(dy.t(), x)),
        "mm(dyT,x)": t(lambda: torch.mm(dy.t(), x)),
        "mm(xT,dy)": t(lambda: torch.mm(x.t(), dy)),
        "addmm_T(xT,dy)": t(lambda: gwt.addmm_(x.t(), dy)),
        "mm(dyT.cont,x)": t(lambda: torch.mm(dy.t().contiguous(), x)),
        "kfa_wgrad": t(lambda: wgrad_into(x, dy, gw, 1, 1, M, K, 1, M, N, 1, 1, 1, 0, True)),
    }
    print(M, N, K, " | ".join(f"{k} {fl / v / 1e9:.0f}" for k, v in res.items()), flush=True)
