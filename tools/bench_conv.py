"""Per-layer timing: hand-written implicit GEMM vs PyTorch/MIOpen, ResNet-50 shapes (bs 256)."""
import os
import sys

import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.conv import conv_fwd, conv_dgrad, wgrad_into  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
torch.backends.cudnn.benchmark = True
SH = [  # Cin, H, Cout, k, stride, pad, count in RN50
    (64, 56, 64, 1, 1, 0, 1), (64, 56, 64, 3, 1, 1, 3), (64, 56, 256, 1, 1, 0, 4), (256, 56, 64, 1, 1, 0, 2),
    (256, 56, 128, 1, 1, 0, 1), (128, 56, 128, 3, 2, 1, 1), (128, 28, 512, 1, 1, 0, 4), (256, 56, 512, 1, 2, 0, 1),
    (512, 28, 128, 1, 1, 0, 3), (128, 28, 128, 3, 1, 1, 3), (512, 28, 256, 1, 1, 0, 1), (256, 28, 256, 3, 2, 1, 1),
    (256, 14, 1024, 1, 1, 0, 6), (512, 28, 1024, 1, 2, 0, 1), (1024, 14, 256, 1, 1, 0, 5), (256, 14, 256, 3, 1, 1, 5),
    (1024, 14, 512, 1, 1, 0, 1), (512, 14, 512, 3, 2, 1, 1), (512, 7, 2048, 1, 1, 0, 3), (1024, 14, 2048, 1, 2, 0, 1),
    (2048, 7, 512, 1, 1, 0, 2), (512, 7, 512, 3, 1, 1, 2),
]
d = torch.device("cuda")


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


tot = {"ours_f": 0, "torch_f": 0, "ours_d": 0, "torch_d": 0, "ours_w": 0, "torch_w": 0}
for (Cin, H, Cout, k, s, p, cnt) in SH:
    x = torch.randn(B, Cin, H, H, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = F.conv2d(x, w, None, s, p)
    dy = torch.randn_like(y)
    flops = 2 * y.numel() * Cin * k * k
    # floor = max(HBM bytes at 5 TB/s, FLOPs at 2 PF/s) for x + y (+ w) moved once
    byts = 2 * (x.numel() + y.numel() + w.numel())
    floor = max(byts / 5e9, flops / 2e12)
    of = t(lambda: conv_fwd(x, w, s, p))
    tf = t(lambda: F.conv2d(x, w, None, s, p))
    od = t(lambda: conv_dgrad(dy, w, x.shape, s, p))
    td = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False,
                                                          [0, 0], 1, [True, False, False]))
    tw = t(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False,
                                                          [0, 0], 1, [False, True, False]))
    gw = torch.zeros_like(w)
    P_, Q_ = y.shape[2], y.shape[3]
    ow = t(lambda: wgrad_into(x, dy, gw, B, H, H, Cin, P_, Q_, Cout, k, k, s, p, True))
    for k_, v in (("ours_f", of), ("torch_f", tf), ("ours_d", od), ("torch_d", td), ("ours_w", ow), ("torch_w", tw)):
        tot[k_] += v * cnt
    tot["floor"] = tot.get("floor", 0) + 3 * floor * cnt
    print(f"Cin{Cin:5d} H{H:3d} Cout{Cout:5d} k{k} s{s} x{cnt}: floor {floor:.3f} | fwd ours {of:.3f}ms ({flops/of/1e9:.0f} TF) "
          f"torch {tf:.3f}ms ({flops/tf/1e9:.0f} TF) | dgrad ours {od:.3f} torch {td:.3f} | wgrad ours {ow:.3f} "
          f"torch {tw:.3f}",
          flush=True)
print("TOTAL (x count) ms:", {k: round(v, 2) for k, v in tot.items()})
