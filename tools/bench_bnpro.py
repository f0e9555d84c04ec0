"""BatchNorm-apply + ReLU folded into the consuming conv (kfa_conv_igemm_bnpro) vs
the separate apply pass + conv, per ResNet-50 bn1->conv2 / bn2->conv3 shape (bs 256).

    python tools/bench_bnpro.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
from kubeflow_controller_amd.ops import conv as convmod  # noqa: E402

SHAPES = [  # C, H, Co, k, count in ResNet-50
    (64, 56, 64, 3, 3), (128, 28, 128, 3, 3), (256, 14, 256, 3, 5), (512, 7, 512, 3, 2),
    (64, 56, 256, 1, 3), (128, 28, 512, 1, 4), (256, 14, 1024, 1, 6), (512, 7, 2048, 1, 3),
]


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
    convmod.TUNE = False
    d = torch.device("cuda")
    N = 256
    tot = [0.0, 0.0, 0.0]
    for C, H, Co, k, cnt in SHAPES:
        pad = k // 2
        x = torch.randn(N, C, H, H, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, k, k, device=d) / (C * k * k) ** 0.5).to(torch.bfloat16)
        w = w.contiguous(memory_format=torch.channels_last)
        g, b = torch.rand(C, device=d) + 0.5, torch.randn(C, device=d) * 0.1
        rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
        ws = torch.empty(3 * C, device=d)
        y = torch.empty_like(x)
        stats = torch.zeros(_lib.lib().kfa_bn_slot_floats(Co), device=d)
        M = N * H * H
        st = _lib.stream()

        def sep():
            _lib.call("kfa_bn_fwd_eval", _lib.ptr(x), None, _lib.ptr(y), _lib.ptr(g), _lib.ptr(b), _lib.ptr(rm),
                      _lib.ptr(rv), _lib.ptr(ws), M, C, 1e-5, 1, st)
            convmod.conv_fwd(y, w, 1, pad, stats)

        def apply_only():
            _lib.call("kfa_bn_fwd_eval", _lib.ptr(x), None, _lib.ptr(y), _lib.ptr(g), _lib.ptr(b), _lib.ptr(rm),
                      _lib.ptr(rv), _lib.ptr(ws), M, C, 1e-5, 1, st)

        ss = ws[:2 * C]
        t_sep = min(timeit(sep) for _ in range(3))
        t_app = min(timeit(apply_only) for _ in range(3))
        t_pro = min(timeit(lambda: convmod.conv_fwd_bnpro(x, ss, w, 1, pad, stats, y)) for _ in range(3))
        stats.zero_()
        tot[0] += t_sep * cnt
        tot[1] += t_pro * cnt
        tot[2] += t_app * cnt
        print(f"C {C:4d} H {H:3d} Co {Co:5d} k{k} x{cnt}: apply+conv {t_sep:7.1f} us (apply {t_app:6.1f}, conv "
              f"{t_sep - t_app:6.1f}) | fused {t_pro:7.1f} us  -> {t_sep - t_pro:+6.1f} us/call", flush=True)
    print(f"TOTAL x count: apply+conv {tot[0] / 1e3:.3f} ms (apply {tot[2] / 1e3:.3f}) | fused {tot[1] / 1e3:.3f} ms",
          flush=True)


if __name__ == "__main__":
    main()
