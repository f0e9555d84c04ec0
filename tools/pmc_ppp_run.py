"""Runs the per-tile ping-pong main-loop probe and gemm_ppp (no-store probe, one
tile per block, and persistent) a few times each for a rocprofv3 --pmc pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402

d = torch.device("cuda")
M, N, K = 32768, 3072, 768
x = torch.randn(M, K, device=d).to(torch.bfloat16)
w = torch.randn(N, K, device=d).to(torch.bfloat16)
for _ in range(3):
    G.gemm_nt(x, w, persistent=7)
    G.gemm_ppp(x, w, blocks=1536, probe=1)
    G.gemm_ppp(x, w, probe=1)
torch.cuda.synchronize()
print("ok")
