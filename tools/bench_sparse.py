"""Owner-side sparse Adam at the Wide&Deep BASELINE shape on 1x MI355X: 65536
examples x 26 fields = 1.70 M looked-up rows of 72 fp32 (64 deep + 8 wide),
Criteo-like power-law ids over the 22.9 M-row table.  Segment-reduce kernels
(default) vs the scatter-add + atomic-exchange kernels (KFA_SPARSE_ATOMIC=1),
interleaved in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.models.wide_deep import WideDeepConfig, synthetic_batch  # noqa: E402
from kubeflow_controller_amd.parallel.embedding import ShardedEmbedding  # noqa: E402


def main():
    cfg = WideDeepConfig()
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    offs = torch.tensor([0] + list(cfg.cardinalities[:-1])).cumsum(0)
    _, ids, _ = synthetic_batch(cfg, batch, generator=torch.Generator().manual_seed(0))
    ids = (ids + offs).reshape(-1).cuda()
    rows = sum(cfg.cardinalities)
    emb = ShardedEmbedding(rows, cfg.row_width, device="cuda")
    g = (torch.randn(ids.numel(), cfg.row_width, device="cuda") * 1e-3).to(torch.bfloat16)
    uniq = torch.unique(ids).numel()
    print(f"n {ids.numel()} unique rows {uniq} ({uniq / ids.numel():.1%}) dim {cfg.row_width}", flush=True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for rnd in range(3):
        for name, atomic in (("segment", "0"), ("atomic", "1")):
            os.environ["KFA_SPARSE_ATOMIC"] = atomic
            for _ in range(2):
                emb.apply_sparse(ids, g)
            torch.cuda.synchronize()
            s.record()
            for _ in range(10):
                emb.apply_sparse(ids, g)
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(s.elapsed_time(e) / 10)
    print(" | ".join(f"{k} {min(v):.3f} ms" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
