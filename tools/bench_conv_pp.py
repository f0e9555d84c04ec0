"""Per-layer A/B of the implicit-GEMM tile variants on the ResNet-50 shapes (bs 256):
128x128 (variant 0 / narrow 1), old 8-wave 256x256 (2), ping-pong 256x256 (4) — forward
(with fused BN statistics, as in the step) and data gradient; numerics vs variant 0."""
import os
import sys

import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib, conv as convmod  # noqa: E402

B = int(os.environ.get("BS", "256"))
SH = [  # Cin, H, Cout, k, stride, pad, count in RN50
    (64, 56, 64, 1, 1, 0, 1), (64, 56, 64, 3, 1, 1, 3), (64, 56, 256, 1, 1, 0, 4), (256, 56, 64, 1, 1, 0, 2),
    (256, 56, 128, 1, 1, 0, 1), (128, 56, 128, 3, 2, 1, 1), (128, 28, 512, 1, 1, 0, 4), (256, 56, 512, 1, 2, 0, 1),
    (512, 28, 128, 1, 1, 0, 3), (128, 28, 128, 3, 1, 1, 3), (512, 28, 256, 1, 1, 0, 1), (256, 28, 256, 3, 2, 1, 1),
    (256, 14, 1024, 1, 1, 0, 6), (512, 28, 1024, 1, 2, 0, 1), (1024, 14, 256, 1, 1, 0, 5), (256, 14, 256, 3, 1, 1, 5),
    (1024, 14, 512, 1, 1, 0, 1), (512, 14, 512, 3, 2, 1, 1), (512, 7, 2048, 1, 1, 0, 3), (1024, 14, 2048, 1, 2, 0, 1),
    (2048, 7, 512, 1, 1, 0, 2), (512, 7, 512, 3, 1, 1, 2),
]
d = torch.device("cuda")
VARS = [int(v) for v in os.environ.get("VARS", "-1,4,6").split(",")]


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


convmod.PP = "0"  # forced variants only: no per-shape routing inside the timed calls
orig = convmod._variant
tot = {}
for (Cin, H, Cout, k, s, p, cnt) in SH:
    x = torch.randn(B, Cin, H, H, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y0 = F.conv2d(x, w, None, s, p)
    dy = torch.randn_like(y0)
    flops = 2 * y0.numel() * Cin * k * k
    stats = torch.zeros(_lib.lib().kfa_bn_slot_floats(Cout), dtype=torch.float32, device=d)
    row = f"Cin{Cin:5d} H{H:3d} Cout{Cout:5d} k{k} s{s} x{cnt}:"
    ref_f = ref_d = None
    for v in VARS:
        convmod._variant = (lambda vv: (lambda M, N, K=0, addend=False: vv if (vv < 4 or (K > 0 and N >= (256 if vv == 4 else 128))) else orig(M, N, K, addend)))(v) \
            if v >= 0 else orig
        yf = convmod.conv_fwd(x, w, s, p, stats)
        dx = convmod.conv_dgrad(dy, w, x.shape, s, p)
        if ref_f is None:
            ref_f, ref_d = yf.float(), dx.float()
            ef = ed = 0.0
        else:
            ef = (yf.float() - ref_f).abs().max().item() / max(1e-6, ref_f.abs().max().item())
            ed = (dx.float() - ref_d).abs().max().item() / max(1e-6, ref_d.abs().max().item())
        tf = t(lambda: convmod.conv_fwd(x, w, s, p, stats))
        td = t(lambda: convmod.conv_dgrad(dy, w, x.shape, s, p))
        stats.zero_()
        tot[(v, "f")] = tot.get((v, "f"), 0) + tf * cnt
        tot[(v, "d")] = tot.get((v, "d"), 0) + td * cnt
        row += f" | v{v} fwd {tf:.3f} ({flops / tf / 1e9:.0f} TF) dgrad {td:.3f} ({flops / td / 1e9:.0f} TF) err {ef:.1e}/{ed:.1e}"
    convmod._variant = orig
    print(row, flush=True)
print("TOTAL ms (x count):", {f"v{k[0]}{k[1]}": round(v, 3) for k, v in sorted(tot.items())}, flush=True)
