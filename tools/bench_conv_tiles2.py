"""Per-shape tile choice for the implicit-GEMM conv over every ResNet-50 (bs 256)
layer: 128x128 (variant 0, 4 waves, 2 blocks/CU), 256x256 (2), 128x256 (4) and
256x128 (5) (8 waves, 1 block/CU) — forward with fused BN statistics and data
gradient with fused BN-backward statistics.  Prints per-shape ms / TFLOP/s and
the step-weighted totals of "always 0", "current rule" and "best per shape"."""
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import conv  # noqa: E402
from kubeflow_controller_amd.ops.batchnorm import bn_slot_workspace  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SH = [  # Cin, H, Cout, k, stride, pad, count in RN50
    (64, 56, 64, 1, 1, 0, 1), (64, 56, 64, 3, 1, 1, 3), (64, 56, 256, 1, 1, 0, 4), (256, 56, 64, 1, 1, 0, 2),
    (256, 56, 128, 1, 1, 0, 1), (128, 56, 128, 3, 2, 1, 1), (128, 28, 512, 1, 1, 0, 4), (256, 56, 512, 1, 2, 0, 1),
    (512, 28, 128, 1, 1, 0, 3), (128, 28, 128, 3, 1, 1, 3), (512, 28, 256, 1, 1, 0, 1), (256, 28, 256, 3, 2, 1, 1),
    (256, 14, 1024, 1, 1, 0, 6), (512, 28, 1024, 1, 2, 0, 1), (1024, 14, 256, 1, 1, 0, 5), (256, 14, 256, 3, 1, 1, 5),
    (1024, 14, 512, 1, 1, 0, 1), (512, 14, 512, 3, 2, 1, 1), (512, 7, 2048, 1, 1, 0, 3), (1024, 14, 2048, 1, 2, 0, 1),
    (2048, 7, 512, 1, 1, 0, 2), (512, 7, 512, 3, 1, 1, 2),
]
d = torch.device("cuda")


def t(fn, it=15):
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


def ok(v, N):
    return v == 0 or (v in (2, 4) and N % 256 == 0) or (v == 5 and N % 128 == 0)


def with_variant(v, fn):
    orig = conv._variant
    conv._variant = (lambda M, N, K=0, addend=False: v if (N > 64 and ok(v, N)) else orig(M, N, K, addend))
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


VS = (0, 2, 4, 5)
tot = {k: 0.0 for k in ("f_rule", "f_best", "g_rule", "g_best")}
for (Cin, H, Cout, k, s, p, cnt) in SH:
    x = torch.randn(B, Cin, H, H, device=d, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=d) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv.conv_fwd(x, w, s, p)
    dy = torch.randn_like(y)
    flops = 2 * y.numel() * Cin * k * k
    row = f"Cin{Cin:5d} H{H:3d} Cout{Cout:5d} k{k} s{s} x{cnt}:"
    if Cout > 64:
        st = bn_slot_workspace(Cout, d)
        rule = t(lambda: conv.conv_fwd(x, w, s, p, st))
        res = {v: with_variant(v, lambda: conv.conv_fwd(x, w, s, p, st)) for v in VS if ok(v, Cout)}
        st.zero_()
        bv = min(res, key=res.get)
        tot["f_rule"] += rule * cnt
        tot["f_best"] += min(rule, res[bv]) * cnt
        row += f" fwd rule {rule:.3f} | " + " ".join(f"v{v} {res[v]:.3f}" for v in res) + f" -> v{bv} ({flops / res[bv] / 1e9:.0f} TF)"
    if Cin > 64:
        link = Link(x, Cin)
        st = bn_slot_workspace(Cin, d)
        rule = t(lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link))
        res = {v: with_variant(v, lambda: conv.conv_dgrad(dy, w, x.shape, s, p, bn=link)) for v in VS if ok(v, Cin)}
        st.zero_()
        bv = min(res, key=res.get)
        tot["g_rule"] += rule * cnt
        tot["g_best"] += min(rule, res[bv]) * cnt
        row += f" || dgrad rule {rule:.3f} | " + " ".join(f"v{v} {res[v]:.3f}" for v in res) + f" -> v{bv}"
    print(row, flush=True)
print({k: round(v, 3) for k, v in tot.items()})
