"""A/B of the ResNet stem (7x7/s2/p3, 3 -> 64 channels, bs 256): MIOpen forward +
the BatchNorm's own statistics pass + MIOpen weight gradient, against the
space-to-depth path on the implicit-GEMM kernels (fused statistics) — same
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
from kubeflow_controller_amd.ops.batchnorm import bn_slot_workspace  # noqa: E402
from kubeflow_controller_amd.ops.conv import conv_fwd, conv_wgrad_vendor, stem_inputs, wgrad_into  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
d = torch.device("cuda")
torch.backends.cudnn.benchmark = True
x = torch.randn(B, 3, 224, 224, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device=d) * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(B, 64, 112, 112, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
slots = bn_slot_workspace(64, d)


def t(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def vendor_fwd():
    y = F.conv2d(x, w, None, 2, 3)
    _lib.call("kfa_bn_stats_partial", _lib.ptr(y), _lib.ptr(slots), y.numel() // 64, 64, _lib.stream())


def ours_fwd():
    xs, ws = stem_inputs(x, w, 3)
    conv_fwd(xs, ws, 1, 0, slots)


xs, ws = stem_inputs(x, w, 3)
dws = torch.empty(64, 4, 4, 16, device=d)
gw = torch.zeros_like(w)


def ours_wgrad():
    wgrad_into(xs, dy, dws, B, 115, 115, 16, 112, 112, 64, 4, 4, 1, 0, accumulate=False)
    _lib.call("kfa_stem_wgrad_fold", _lib.ptr(dws), _lib.ptr(gw), 0, 1, 64, 7, 7, 3, _lib.stream())


def vendor_wgrad():
    gw.add_(conv_wgrad_vendor(x, dy, w, 2, 3))


res = {k: [] for k in ("vendor_fwd", "ours_fwd", "s2d_only", "vendor_wgrad", "ours_wgrad")}
for _ in range(3):
    res["vendor_fwd"].append(t(vendor_fwd))
    res["ours_fwd"].append(t(ours_fwd))
    res["s2d_only"].append(t(lambda: stem_inputs(x, w, 3)))
    res["vendor_wgrad"].append(t(vendor_wgrad))
    res["ours_wgrad"].append(t(ours_wgrad))
slots.zero_()
for k, v in res.items():
    print(f"{k:14s} median {sorted(v)[1]:.3f} ms  (min {min(v):.3f})")
