"""Run one hot op a few times on its production shape, for rocprofv3 --pmc passes.

    rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY ... --output-format csv -d out -o x -- python tools/probe_kernels.py wgrad_bert

Ops: wgrad_bert (dW [3072, 768] of a 32768-token FFN-up), attn_bwd / attn_fwd
(BERT-base, 256 x 128 tokens), conv_fwd_3x3_14 / conv_dgrad_3x3_14 (ResNet-50
stage 4, 256 ch, bs 256), gemm_nt (32768 x 3072 x 768).
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(op: str, iters: int = 5) -> None:
    d = torch.device("cuda")
    torch.manual_seed(0)
    bf = lambda *s: torch.randn(*s, device=d).to(torch.bfloat16)  # noqa: E731
    if op == "wgrad_bert":
        from kubeflow_controller_amd.ops.conv import wgrad_into
        x, dy = bf(32768, 768), bf(32768, 3072)
        gw = torch.zeros(3072, 768, device=d, dtype=torch.float32)
        fn = lambda: wgrad_into(x, dy, gw, 1, 1, 32768, 768, 1, 32768, 3072, 1, 1, 1, 0, True)  # noqa: E731
    elif op in ("attn_fwd", "attn_bwd"):
        from kubeflow_controller_amd.ops import transformer as T
        B, S, h = 256, 128, 12
        qkv, bqkv, kb = bf(B * S, 3 * h * 64), torch.randn(3 * h * 64, device=d) * 0.1, torch.zeros(B, S, device=d)
        out, lse = T.attn_fwd(qkv, bqkv, kb, B, S, h, 0.1, 1)
        dout, db = bf(B * S, h * 64), torch.zeros(3 * h * 64, device=d)
        fn = (lambda: T.attn_fwd(qkv, bqkv, kb, B, S, h, 0.1, 1)) if op == "attn_fwd" else \
            (lambda: T.attn_bwd(qkv, bqkv, kb, out, lse, dout, db, B, S, h, 0.1, 1))
    elif op.startswith("conv_"):
        # conv_fwd_3x3_14 (legacy name) or conv_{fwd,dgrad,wgrad}_<Cin>_<H>_<Cout>_<k>_<stride>
        from kubeflow_controller_amd.ops.conv import conv_dgrad, conv_fwd
        parts = op.split("_")
        if len(parts) == 7:
            cin, hh, cout, k, st = (int(v) for v in parts[2:])
        else:
            cin, hh, cout, k, st = 256, 14, 256, 3, 1
        pad = k // 2
        ho = (hh + 2 * pad - k) // st + 1
        x = bf(256, cin, hh, hh).contiguous(memory_format=torch.channels_last)
        w = (bf(cout, cin, k, k) * 0.05).contiguous(memory_format=torch.channels_last)
        dy = bf(256, cout, ho, ho).contiguous(memory_format=torch.channels_last)
        if "wgrad" in op:  # conv_wgrad_<Cin>_<H>_<Cout>_<k>_<stride>: dW into a bf16 gradient
            from kubeflow_controller_amd.ops.conv import wgrad_into
            gw = torch.zeros_like(w)
            fn = lambda: wgrad_into(x, dy, gw, 256, hh, hh, cin, ho, ho, cout, k, k, st, pad, True)  # noqa: E731
        else:
            fn = (lambda: conv_fwd(x, w, st, pad)) if "fwd" in op else (lambda: conv_dgrad(dy, w, x.shape, st, pad))
    elif op == "gemm_nt":
        from kubeflow_controller_amd.ops import gemm as G
        a, b = bf(32768, 768), bf(3072, 768)
        fn = lambda: G.gemm_nt(a, b)  # noqa: E731
    else:
        raise SystemExit(f"unknown op {op}")
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print(f"{op}: {iters} runs ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
