"""Time the small-table embedding gradient (BERT position / segment tables,
32768 tokens x 768): kfa_embed_small_bwd vs the one-hot GEMM path.

    python tools/bench_embed_small.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import transformer as T  # noqa: E402


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
    n, D = 32768, 768
    dy = torch.randn(n, D, device=d).to(torch.bfloat16)
    for name, R, ids in (("positions", 512, torch.arange(128, device=d).repeat(n // 128)),
                         ("segments", 2, (torch.rand(n, device=d) < 0.4).long())):
        t = torch.randn(R, D, device=d).requires_grad_()
        res = {}
        for small in (True, False):
            T.EMB_SMALL_KERNEL = small

            def step():
                t.grad = None
                T.embedding_sum([t], [ids]).backward(dy)
            res[small] = min(timeit(step) for _ in range(3))
        fwd = min(timeit(lambda: T.embedding_sum([t], [ids])) for _ in range(3))
        print(f"embed small-table {name:9s} R={R}: fwd {fwd:6.1f} us | fwd+bwd small kernel {res[True]:6.1f} us, "
              f"one-hot GEMM {res[False]:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
