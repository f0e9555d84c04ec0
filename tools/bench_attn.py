"""BERT-base attention (256 x 128 tokens, 12 heads, dropout 0.1) fwd / bwd timing.

    python tools/bench_attn.py

Prints one line: fwd (with / without writing the packed keep mask), bwd (from the
mask / re-hashing / without the bias gradient / no dropout) in us per call, and a
checksum of the outputs (the same seed gives bit-identical outputs across kernel
forms: compare the lines).
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
    p = 0.1
    qkv = torch.randn(B * S, 3 * h * 64, device=d).to(torch.bfloat16)
    bqkv = torch.randn(3 * h * 64, device=d) * 0.1
    kb = torch.zeros(B, S, device=d)
    kb[:, 100:] = -10000.0
    dout = torch.randn(B * S, h * 64, device=d).to(torch.bfloat16)
    out, lse, mask = T.attn_fwd(qkv, bqkv, kb, B, S, h, p, 7, want_mask=True)
    db = torch.zeros(3 * h * 64, device=d)
    dq = T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, h, p, 7, mask=mask)
    csum = (out.float().abs().sum().item(), lse.sum().item(), dq.float().abs().sum().item(), db.abs().sum().item())
    best = lambda fn: min(timeit(fn) for _ in range(3))  # noqa: E731
    tfm = best(lambda: T.attn_fwd(qkv, bqkv, kb, B, S, h, p, 7, want_mask=True))
    tf = best(lambda: T.attn_fwd(qkv, bqkv, kb, B, S, h, p, 7))
    tf0 = best(lambda: T.attn_fwd(qkv, bqkv, kb, B, S, h, 0.0, 7))
    tbm = best(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, None, B, S, h, p, 7, mask=mask))
    tbh = best(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, None, B, S, h, p, 7))
    tbb = best(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, h, p, 7, mask=mask))
    tb0 = best(lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, None, B, S, h, 0.0, 7))
    print(f"attn fwd {tfm:6.1f} us (mask) {tf:6.1f} (no mask) {tf0:6.1f} (p=0) | bwd {tbm:6.1f} us (mask) "
          f"{tbh:6.1f} (re-hash) {tbb:6.1f} (mask + bias atomics) {tb0:6.1f} (p=0) | fwd+bwd {tfm + tbm:6.1f} us/layer | "
          f"checksum out {csum[0]:.6e} lse {csum[1]:.6e} dqkv {csum[2]:.6e} dbias {csum[3]:.6e}", flush=True)


if __name__ == "__main__":
    main()
