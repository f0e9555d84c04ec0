"""BERT FFN-down data gradient + GELU backward + FFN-up bias gradient:
hipBLASLt / own GEMM + the bias_act_bwd pass vs the fused gemm_ppw_dact (one GEMM launch
+ a small column-sum reduce).  bs 256 x 128 tokens.

    python tools/bench_dact.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops.transformer import bias_act_bwd  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000


def main():
    d = torch.device("cuda")
    for T, H, F in ((32768, 768, 3072), (16384, 1024, 4096)):
        df2 = torch.randn(T, H, device=d).to(torch.bfloat16)
        w2 = (torch.randn(H, F, device=d) / F ** 0.5).to(torch.bfloat16)  # [out = H, in = F]
        w2t = w2.t().contiguous()
        z = torch.randn(T, F, device=d).to(torch.bfloat16)
        b1 = torch.randn(F, device=d) * 0.1
        db = torch.zeros(F, device=d)
        res = {
            "hipblaslt+pass": lambda: bias_act_bwd(torch.mm(df2, w2), z, b1, "gelu", db),
            "ppw+pass": lambda: bias_act_bwd(G.gemm_ppp(df2, w2t, probe=9, split=False), z, b1, "gelu", db),
            "gemm only (hipblaslt)": lambda: torch.mm(df2, w2),
            "pass only": lambda: bias_act_bwd(df2.new_empty(T, F), z, b1, "gelu", db),
            "fused ppw-dact": lambda: G.gemm_ppw_dact(df2, w2t, z, b1, db),
            "fused ppw-dact-nt": lambda: G.gemm_ppw_dact(df2, w2t, z, b1, db, nt=True),
        }
        out = {k: min(timeit(f) for _ in range(3)) for k, f in res.items()}
        print(f"T {T} H {H} F {F}: " + " | ".join(f"{k} {v:7.1f} us" for k, v in out.items()), flush=True)


if __name__ == "__main__":
    main()
