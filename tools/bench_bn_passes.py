"""Per-pass BatchNorm kernel rates on the ResNet-50 bs-256 block-output shapes, 1x MI355X,
against PyTorch's own 2-read / 1-write bf16 elementwise kernel (``torch.add(out=)``) on
the same bytes as the attainable streaming rate.

  fwd3   kfa_bn_fwd_train_prestats, residual + ReLU + bit mask  (bn_apply<t,t,t,f>):
         reads x, res; writes y, bits                 6.125 B / element
  bwd3   kfa_bn_bwd_prestats, mask from the bits, no dres        (bn_bwd_apply<3,false>):
         reads dy, x, bits; writes dx                 6.125 B / element
  bwd2   kfa_bn_bwd_prestats, mask recomputed from x and ss      (bn_bwd_apply<2,false>):
         reads dy, x; writes dx                       6 B / element

Each prestats call also runs its finalize (one small launch, a few us).

    python tools/bench_bn_passes.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
from kubeflow_controller_amd.ops import batchnorm as BN  # noqa: E402,F401  (registers the entry points)


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    d = torch.device("cuda")
    L = _lib.lib()
    print("| shape (M x C) | pass | us | TB/s | torch.add us | torch.add TB/s |")
    print("|---|---|---:|---:|---:|---:|")
    for HW, C in [(56, 256), (28, 512), (14, 1024), (7, 2048), (56, 64), (28, 128), (14, 256), (7, 512)]:
        M = 256 * HW * HW
        n = M * C
        g = torch.Generator(device=d).manual_seed(0)
        x = torch.randn(M, C, device=d, generator=g).to(torch.bfloat16)
        r = torch.randn(M, C, device=d, generator=g).to(torch.bfloat16)
        dy = torch.randn(M, C, device=d, generator=g).to(torch.bfloat16)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        mb = torch.empty(n // 8, dtype=torch.uint8, device=d)
        w, b = torch.ones(C, device=d), torch.zeros(C, device=d)
        rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
        mean, inv = torch.zeros(C, device=d), torch.ones(C, device=d)
        dg, db = torch.zeros(C, device=d), torch.zeros(C, device=d)
        slots = torch.zeros(L.kfa_bn_slot_floats(C), device=d)
        coef = torch.zeros(L.kfa_bn_coef_floats(C), device=d)
        ss = torch.cat([torch.ones(C, device=d), torch.zeros(C, device=d)])
        st = _lib.stream()

        def fwd3():
            _lib.call("kfa_bn_fwd_train_prestats", _lib.ptr(x), _lib.ptr(r), _lib.ptr(y), _lib.ptr(w), _lib.ptr(b),
                      _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(mean), _lib.ptr(inv), _lib.ptr(slots), _lib.ptr(coef),
                      M, C, 1e-5, 0.1, 1, _lib.ptr(mb), st)

        def bwd(mm):
            return lambda: _lib.call("kfa_bn_bwd_prestats", _lib.ptr(dy), _lib.ptr(x), None, _lib.ptr(w),
                                     _lib.ptr(mean), _lib.ptr(inv), _lib.ptr(dx), None, _lib.ptr(dg), _lib.ptr(db),
                                     _lib.ptr(slots), _lib.ptr(coef), M, C, 1, 0,
                                     _lib.ptr(ss) if mm == 2 else None, _lib.ptr(mb) if mm == 3 else None, st)
        t_add = timeit(lambda: torch.add(x, r, out=y), a.iters)
        passes = [("fwd3", fwd3, 6.125), ("bwd3", bwd(3), 6.125), ("bwd2", bwd(2), 6.0)]
        for name, fn, bpe in passes:
            t = timeit(fn, a.iters)
            print(f"| {M} x {C} | {name} | {t:.1f} | {bpe * n / t / 1e6:.2f} | {t_add:.1f} | {6 * n / t_add / 1e6:.2f} |",
                  flush=True)


if __name__ == "__main__":
    main()
