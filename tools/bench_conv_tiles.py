"""Per-shape tile choice for the implicit-GEMM conv: 128x128 (4 waves, 2 blocks/CU)
vs 256x256 (8 waves, 1 block/CU) on every ResNet-50 (bs 256) launch whose output
width N is a multiple of 256 — forward with fused BN statistics, data gradient
with fused BN-backward statistics (the step's epilogues)."""
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib, conv  # noqa: E402
from kubeflow_controller_amd.ops.batchnorm import bn_slot_workspace  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SH = [  # Cin, H, Cout, k, stride, pad, count in RN50 (bench_conv.py)
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


def with_variant(v, fn):
    orig = conv._variant
    conv._variant = (lambda M, N, K=0: v if (N % 256 == 0 and v == 2) else orig(M, N, K))
    try:
        return t(fn)
    finally:
        conv._variant = orig


class Link:  # the BnBwdLink fields conv_dgrad reads
    def __init__(self, x, C):
        self.x, self.y, self.relu, self.mb = x, None, True, None
        self.mean = torch.zeros(C, device=d)
        self.ss = torch.cat([torch.ones(C, device=d), torch.zeros(C, device=d)])
        self.prestats = False


tot = {"fwd0": 0.0, "fwd2": 0.0, "dg0": 0.0, "dg2": 0.0}
for (Cin, H, Cout, k, s, p, cnt) in SH:
    x = torch.randn(B, Cin, H, H, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv.conv_fwd(x, w, s, p)
    dy = torch.randn_like(y)
    flops = 2 * y.numel() * Cin * k * k
    row = f"Cin{Cin:5d} H{H:3d} Cout{Cout:5d} k{k} s{s} x{cnt}:"
    if Cout % 256 == 0:
        st = bn_slot_workspace(Cout, d)
        f0 = with_variant(0, lambda: conv.conv_fwd(x, w, s, p, st))
        f2 = with_variant(2, lambda: conv.conv_fwd(x, w, s, p, st))
        st.zero_()
        tot["fwd0"] += f0 * cnt
        tot["fwd2"] += min(f0, f2) * cnt
        row += f" fwd+stats 128x128 {f0:.3f} ({flops / f0 / 1e9:.0f} TF) 256x256 {f2:.3f} ({flops / f2 / 1e9:.0f} TF)"
    if Cin % 256 == 0:
        link = Link(x, Cin)
        st = bn_slot_workspace(Cin, d)
        g0 = with_variant(0, lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link))
        g2 = with_variant(2, lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link))
        st.zero_()
        tot["dg0"] += g0 * cnt
        tot["dg2"] += min(g0, g2) * cnt
        row += f" | dgrad+bnstats 128x128 {g0:.3f} ({flops / g0 / 1e9:.0f} TF) 256x256 {g2:.3f} ({flops / g2 / 1e9:.0f} TF)"
    print(row, flush=True)
print("TOTAL (x count, best-of per shape) ms:", {k: round(v, 3) for k, v in tot.items()})

# N <= 64 launches: 128x64 (4 waves of 32x64, 3 blocks/CU) vs 256x64 (4 waves of 64x64, 2 blocks/CU)
def with_narrow(v, fn):
    orig = conv.NARROW
    conv.NARROW = v
    try:
        return t(fn)
    finally:
        conv.NARROW = orig


nt = {"n1": 0.0, "n3": 0.0, "best": 0.0}
for (Cin, H, Cout, k, s, p, cnt) in SH:
    x = torch.randn(B, Cin, H, H, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv.conv_fwd(x, w, s, p)
    dy = torch.randn_like(y)
    row = f"Cin{Cin:5d} H{H:3d} Cout{Cout:5d} k{k} s{s} x{cnt}:"
    if Cout <= 64:
        st = bn_slot_workspace(Cout, d)
        a = with_narrow(1, lambda: conv.conv_fwd(x, w, s, p, st))
        b = with_narrow(3, lambda: conv.conv_fwd(x, w, s, p, st))
        st.zero_()
        nt["n1"] += a * cnt
        nt["n3"] += b * cnt
        nt["best"] += min(a, b) * cnt
        row += f" fwd+stats K={Cin * k * k}: 128x64 {a:.3f} 256x64 {b:.3f}"
    if Cin <= 64:
        link = Link(x, Cin)
        st = bn_slot_workspace(Cin, d)
        a = with_narrow(1, lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link))
        b = with_narrow(3, lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link))
        st.zero_()
        nt["n1"] += a * cnt
        nt["n3"] += b * cnt
        nt["best"] += min(a, b) * cnt
        row += f" | dgrad+bnstats K={Cout * k * k}: 128x64 {a:.3f} 256x64 {b:.3f}"
    if Cout <= 64 or Cin <= 64:
        print(row, flush=True)
print("NARROW TOTAL (x count) ms:", {k: round(v, 3) for k, v in nt.items()})
