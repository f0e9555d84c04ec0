"""ResNet-50 stem max pool (3x3/s2/p1 over [256, 64, 112, 112] NHWC bf16): time per
call and achieved HBM bandwidth (bytes the op must move / time), 1x MI355X."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops.pool import _MaxPoolFn  # noqa: E402


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


def main():
    d = torch.device("cuda")
    x = torch.randn(256, 64, 112, 112, device=d).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    y = _MaxPoolFn.apply(x, 3, 2, 1)
    dy = torch.randn_like(y)
    tf = timeit(lambda: _MaxPoolFn.apply(x.detach(), 3, 2, 1))
    tb = timeit(lambda: torch.autograd.grad(y, x, dy, retain_graph=True))
    fb = x.numel() * 2 + y.numel() * 3          # read x, write y + uint8 index
    bb = y.numel() * 3 + x.numel() * 2          # read dy + index, write dx
    print(f"maxpool fwd {tf:.3f} ms ({fb / tf / 1e6:.0f} GB/s)  bwd {tb:.3f} ms ({bb / tb / 1e6:.0f} GB/s)")


if __name__ == "__main__":
    main()
