"""BERT-base attention (256 x 128 tokens, 12 heads, dropout 0.1) fwd / bwd timing.

    KFA_ATTN_PF=0|1 python tools/bench_attn.py     (the env picks the S = 128 kernels)

Prints one line: fwd / bwd us per call and a checksum of the outputs (the same
seed gives bit-identical outputs across kernel forms: compare the lines).
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
    torch.manual_seed(0)
    B, S, h = 256, 128, 12
    qkv = torch.randn(B * S, 3 * h * 64, device=d).to(torch.bfloat16)
    bqkv = torch.randn(3 * h * 64, device=d) * 0.1
    kb = torch.zeros(B, S, device=d)
    kb[:, 100:] = -10000.0
    dout = torch.randn(B * S, h * 64, device=d).to(torch.bfloat16)
    out, lse = T.attn_fwd(qkv, bqkv, kb, B, S, h, 0.1, 7)
    db = torch.zeros(3 * h * 64, device=d)
    dq = T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, h, 0.1, 7)
    dq = dq[0] if isinstance(dq, tuple) else dq
    csum = (out.float().abs().sum().item(), lse.sum().item(), dq.float().abs().sum().item(), db.abs().sum().item())
    tf = min(timeit(lambda: T.attn_fwd(qkv, bqkv, kb, B, S, h, 0.1, 7)) for _ in range(3))
    tb = min(timeit(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, h, 0.1, 7)) for _ in range(3))
    tn = min(timeit(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, None, B, S, h, 0.1, 7)) for _ in range(3))
    print(f"attn PF={os.environ.get('KFA_ATTN_PF', '1')} fwd {tf:7.1f} us  bwd {tb:7.1f} us (no bias grad {tn:7.1f})  "
          f"checksum out {csum[0]:.6e} lse {csum[1]:.6e} dqkv {csum[2]:.6e} dbias {csum[3]:.6e}", flush=True)


if __name__ == "__main__":
    main()
