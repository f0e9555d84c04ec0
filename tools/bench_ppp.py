"""Dense GEMM shapes of BERT-base / W&D / ResNet-FC on 1x MI355X: hipBLASLt
(``torch.mm``) vs the ping-pong kernel (per-tile launch) vs the persistent
ping-pong kernel with the C write overlapped (``gemm_ppp``).  Random bf16
operands, CUDA-event timing, A/B interleaved in one process (rule 24)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import gemm as G  # noqa: E402

SHAPES = [(32768, 2304, 768), (32768, 768, 768), (32768, 3072, 768), (32768, 768, 3072), (32768, 768, 2304),
          (5120, 30528, 768), (5120, 768, 30528), (5120, 768, 768), (256, 1000, 2048), (8192, 8192, 8192)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def stagger_sweep(d, shapes):
    """KFA_PPP_STAGGER=1: odd blocks start late by 0 .. 12 us (the C-burst stagger experiment)."""
    from kubeflow_controller_amd.ops import _lib
    _lib.register("kfa_gemm_ppp_set_stagger", [_lib.I])
    L = _lib.lib()
    for M, N, K in shapes:
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, device=d).to(torch.bfloat16)
        out = []
        for ticks in (0, 300, 600, 900, 1200):
            L.kfa_gemm_ppp_set_stagger(ticks)
            t1 = min(timeit(lambda: G.gemm_ppp(x, w, bn=256, split=False)) for _ in range(3))
            t2 = min(timeit(lambda: G.gemm_ppp(x, w, probe=9, split=False)) for _ in range(3))
            out.append(f"{ticks * 10 / 1000:4.1f}us: ppp {t1 * 1e3:6.1f} ppw {t2 * 1e3:6.1f}")
        L.kfa_gemm_ppp_set_stagger(0)
        th = min(timeit(lambda: torch.mm(x, w.t())) for _ in range(3))
        print(f"stagger {M}x{N}x{K} hipblaslt {th * 1e3:6.1f} | " + " | ".join(out), flush=True)


def main():
    d = torch.device("cuda")
    if os.environ.get("KFA_PPP_STAGGER") == "1":
        stagger_sweep(d, [(32768, 3072, 768), (32768, 768, 3072), (32768, 2304, 768)])
        return
    shapes = SHAPES
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    for M, N, K in shapes:
        x = torch.randn(M, K, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, device=d).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        res = {}
        res.pop("-", None)
        for rnd in range(3):
            for name, fn in (("hipblaslt", lambda: torch.mm(x, w.t())),
                             ("ppp-nosplit", lambda: G.gemm_ppp(x, w, bn=256, split=False)),
                             ("ppp", lambda: G.gemm_ppp(x, w, bn=256)),
                             ("ppp192-4ph", lambda: G.gemm_ppp(x, w, bn=192, probe=7)) if N % 192 == 0 else ("-", lambda: None),
                             ("ppp192", lambda: G.gemm_ppp(x, w, bn=192)) if N % 192 == 0 else ("-", lambda: None),
                             ("ppp192-nost", lambda: G.gemm_ppp(x, w, bn=192, probe=1)) if N % 192 == 0 else ("-", lambda: None),
                             ("ppp-nostore", lambda: G.gemm_ppp(x, w, bn=256, probe=1)),
                             ("ppp-nostore-nosplit", lambda: G.gemm_ppp(x, w, bn=256, probe=1, split=False)),
                             ("ppw", lambda: G.gemm_ppp(x, w, probe=9, split=False)),
                             ("ppw-nt", lambda: G.gemm_ppp(x, w, probe=10, split=False)),
                             *([("skinny", lambda: G.gemm_skinny(x, w))] if M <= 16384 and N % 4 == 0 else []),
                             *([("skinny-s2", lambda: G.gemm_skinny(x, w, splits=2)),
                                ("skinny-s4", lambda: G.gemm_skinny(x, w, splits=4)),
                                ("skinny-s8", lambda: G.gemm_skinny(x, w, splits=8))]
                               if M <= 256 and N % 4 == 0 else [])):
                res.setdefault(name, []).append(timeit(fn))
        ref = torch.mm(x, w.t()).float()
        err = max((G.gemm_ppp(x, w, bn=b).float() - ref).abs().max().item() for b in ((256, 192) if N % 192 == 0 else (256,)))
        err = max(err, (G.gemm_ppp(x, w, probe=9, split=False).float() - ref).abs().max().item())
        res.pop("-", None)
        line = " | ".join(f"{k} {min(v) * 1e3:7.1f} us {fl / min(v) / 1e9:6.0f} TF/s" for k, v in res.items())
        print(f"{M:6d} {N:5d} {K:5d} | {line} | ppp max|err| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
