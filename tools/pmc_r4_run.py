"""Workload for a rocprofv3 --pmc pass over the round-3 kernels (one process,
a few dispatches each): gemm_ppp on the BERT FFN-up shape (256-wide tiles) and
the out-projection (192-wide, three-phase), the split remainder (MLM-decoder
dgrad), wgrad_pp_kernel on the BERT QKV weight gradient, and the segment-reduce
sparse Adam of the Wide&Deep tables (segsparse.hip)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402
from kubeflow_controller_amd.ops.conv import wgrad_into  # noqa: E402

d = torch.device("cuda")
which = sys.argv[1] if len(sys.argv) > 1 else "all"
if which in ("all", "gemm"):
    for M, N, K, bn in ((32768, 3072, 768, 256), (32768, 768, 768, 192), (5120, 768, 30528 // 64 * 64, 256)):
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, device=d).to(torch.bfloat16)
        for _ in range(3):
            G.gemm_ppp(x, w, bn=bn)
if which in ("all", "wgrad"):
    rows, co, ci = 32768, 2304, 768
    x = torch.randn(rows, ci, device=d).to(torch.bfloat16)
    dy = torch.randn(rows, co, device=d).to(torch.bfloat16)
    out = torch.zeros(co, ci, device=d)
    for _ in range(3):
        wgrad_into(x, dy, out, 1, 1, rows, ci, 1, rows, co, 1, 1, 1, 0, accumulate=True)
if which in ("all", "sparse"):
    from kubeflow_controller_amd.models.wide_deep import WideDeepConfig, synthetic_batch
    from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding
    cfg = WideDeepConfig()
    offs = torch.tensor([0] + list(cfg.cardinalities[:-1])).cumsum(0)
    _, ids, _ = synthetic_batch(cfg, 65536, generator=torch.Generator().manual_seed(0))
    ids = (ids + offs).reshape(-1).cuda()
    emb = ShardedEmbedding(sum(cfg.cardinalities), cfg.row_width, device="cuda")
    g = (torch.randn(ids.numel(), cfg.row_width, device="cuda") * 1e-3).to(torch.bfloat16)
    for _ in range(3):
        emb.apply_sparse(ids, g)
torch.cuda.synchronize()
print("ok")
