#!/usr/bin/env python3
"""Time the N = 768 BERT GEMMs (and the other hipBLASLt-routed shapes) on every own
persistent variant vs hipBLASLt, the way ops/routes.py times a decision (median of
3 x 30 launches).  Forward shapes compare torch.mm(a, w.t()); data-gradient shapes
torch.mm(dz, w) (the library's NN form) against the own kernels on the cached
transposed weight."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops.routes import time_ms  # noqa: E402

SHAPES = [("proj", 32768, 768, 3072), ("proj", 32768, 768, 768), ("proj_dgrad", 32768, 768, 2304),
          ("proj_dgrad", 32768, 768, 3072), ("proj_dgrad", 32768, 768, 768), ("proj", 32768, 3072, 768),
          ("dense_fwd", 65536, 512, 1024)]


def main():
    d = torch.device("cuda")
    out = {}
    for kind, M, N, K in SHAPES:
        torch.manual_seed(0)
        if kind == "proj_dgrad":
            dz = torch.randn(M, K, device=d).to(torch.bfloat16)
            w = (torch.randn(K, N, device=d) * 0.05).to(torch.bfloat16)
            wt = w.t().contiguous()
            cands = [("hipblaslt", lambda: torch.mm(dz, w))] + G._ppp_candidates(dz, wt)
        else:
            a = torch.randn(M, K, device=d).to(torch.bfloat16)
            w = (torch.randn(N, K, device=d) * 0.05).to(torch.bfloat16)
            cands = [("hipblaslt", lambda: torch.mm(a, w.t()))] + G._ppp_candidates(a, w)
        t = {n: round(time_ms(f), 5) for n, f in cands}
        best = min((v, n) for n, v in t.items() if n != "hipblaslt")
        key = f"{kind}|{M},{N},{K}"
        out[key] = t
        print(f"{key}: hipblaslt {t['hipblaslt']:.4f}  best own {best[1]} {best[0]:.4f}  "
              f"({(t['hipblaslt'] / best[0] - 1) * 100:+.1f} %)  {t}", flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
