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
ROWS = int(os.environ.get("ROWS", "32768"))  # BERT-base 256 x 128 tokens
for (M, N, K) in [(ROWS, 3072, 768), (ROWS, 2304, 768), (ROWS, 768, 3072), (ROWS, 768, 768)]:
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=d, dtype=torch.bfloat16)
    gwt = torch.zeros(K, N, device=d, dtype=torch.bfloat16)
    gw32 = torch.zeros(N, K, device=d, dtype=torch.float32)  # the flat fp32 gradient bucket (the real target)
    fl = 2 * M * N * K
    res = {
        "addmm_(dyT,x)": t(lambda: gw.addmm_(dy.t(), x)),
        "mm(dyT,x)": t(lambda: torch.mm(dy.t(), x)),
        "mm(xT,dy)": t(lambda: torch.mm(x.t(), dy)),
        "addmm_T(xT,dy)": t(lambda: gwt.addmm_(x.t(), dy)),
        "mm(dyT.cont,x)": t(lambda: torch.mm(dy.t().contiguous(), x)),
        "kfa_wgrad": t(lambda: wgrad_into(x, dy, gw, 1, 1, M, K, 1, M, N, 1, 1, 1, 0, True)),
        "kfa_wgrad_f32": t(lambda: wgrad_into(x, dy, gw32, 1, 1, M, K, 1, M, N, 1, 1, 1, 0, True)),
        "mm+add_f32": t(lambda: gw32.add_(torch.mm(dy.t(), x))),
    }
    print(M, N, K, " | ".join(f"{k} {fl / v / 1e9:.0f}" for k, v in res.items()), flush=True)
