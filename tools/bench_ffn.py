"""BERT FFN-up (32768 x 3072 x 768) forward and its dgrad, hipBLASLt + the
separate epilogue pass vs the hand-written GEMM with the fused epilogue, per
GEMM variant; isolated calls, same process (ms per call)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops import transformer as T  # noqa: E402


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


d = torch.device("cuda")
M, H, I = 32768, 768, 3072
h1 = torch.randn(M, H, device=d).to(torch.bfloat16)
w1 = (torch.randn(I, H, device=d) * 0.05).to(torch.bfloat16)
b1 = torch.randn(I, device=d) * 0.1
w2 = (torch.randn(H, I, device=d) * 0.05).to(torch.bfloat16)
df2 = torch.randn(M, H, device=d).to(torch.bfloat16)
f1 = torch.randn(M, I, device=d).to(torch.bfloat16)
db = torch.zeros(I, device=d)
w2t = G.transpose(w2)
res = {
    "fwd hipBLASLt mm": timeit(lambda: torch.mm(h1, w1.t())),
    "fwd hipBLASLt mm + bias_act_fwd": timeit(lambda: T.bias_act_fwd(torch.mm(h1, w1.t()), b1, "gelu")),
    "bwd hipBLASLt mm": timeit(lambda: torch.mm(df2, w2)),
    "bwd hipBLASLt mm + bias_act_bwd": timeit(lambda: T.bias_act_bwd(torch.mm(df2, w2), f1, b1, "gelu", db)),
}
for v in (0, 3, 4):
    res[f"fwd v{v} plain"] = timeit(lambda: G.gemm_nt(h1, w1, persistent=v))
    res[f"fwd v{v} bias+gelu+z"] = timeit(lambda: G.gemm_nt(h1, w1, bias=b1, act="gelu", want_z=True, persistent=v))
    res[f"fwd v{v} bias+gelu"] = timeit(lambda: G.gemm_nt(h1, w1, bias=b1, act="gelu", persistent=v))
    res[f"bwd v{v} plain"] = timeit(lambda: G.gemm_nt(df2, w2t, persistent=v))
    res[f"bwd v{v} dgelu+dbias"] = timeit(lambda: G.gemm_nt(df2, w2t, zin=f1, dact="gelu", dbias=db, persistent=v))
    res[f"bwd v{v} dgelu"] = timeit(lambda: G.gemm_nt(df2, w2t, zin=f1, dact="gelu", persistent=v))
for k, v in res.items():
    print(f"{k:34s} {v:.3f} ms")
