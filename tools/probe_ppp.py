"""gemm_ppp timing probes at one tile per block (the per-tile launch's geometry):
no-store build with its own loop, pp's loop shape, all-generic k-tiles; vs the
per-tile ping-pong main loop (gemm_pp_kernel probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from tools.bench_ppp import timeit  # noqa: E402

d = torch.device("cuda")
for M, N, K in [(32768, 3072, 768), (32768, 2304, 768), (8192, 8192, 8192)]:
    x = torch.randn(M, K, device=d).to(torch.bfloat16)
    w = torch.randn(N, K, device=d).to(torch.bfloat16)
    tiles = (M // 256) * ((N + 255) // 256)
    out = []
    for _ in range(2):
        for probe in (1, 2, 3):
            t = min(timeit(lambda: G.gemm_ppp(x, w, blocks=tiles, probe=probe)) for _ in range(2))
            out.append(f"probe{probe} {t * 1e3:6.1f}")
        t = min(timeit(lambda: G.gemm_nt(x, w, persistent=7)) for _ in range(2))
        out.append(f"pp-noepi {t * 1e3:6.1f}")
    print(f"{M}x{N}x{K}: " + " | ".join(out), flush=True)
