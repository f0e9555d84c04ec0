"""BatchNorm(+residual)(+ReLU) kernels on ResNet-50 bs-256 shapes: time per call and
achieved HBM bandwidth (bytes the op must move / time), 1x MI355X.

fwd (prestats): y = act(bn(x) [+ res])         reads x [, res], writes y
bwd (prestats): dx [, dres] from dy, x [, y]   reads dy, x [, y], writes dx [, dres]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
from kubeflow_controller_amd.ops import batchnorm as BN  # noqa: E402


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
    for (HW, C) in [(56, 64), (56, 256), (28, 512), (14, 1024), (7, 2048)]:
        M = 256 * HW * HW
        x = torch.randn(M, C, device=d).to(torch.bfloat16)
        res = torch.randn(M, C, device=d).to(torch.bfloat16)
        g, b = torch.ones(C, device=d), torch.zeros(C, device=d)
        rm, rv = torch.zeros(C, device=d), torch.ones(C, device=d)
        for has_res in (False, True):
            r = res if has_res else None
            y = BN.bn_act(x, g, b, rm, rv, r, True, 0.1, 1e-5, True)
            t_f = timeit(lambda: BN.bn_act(x, g, b, rm, rv, r, True, 0.1, 1e-5, True))
            nbytes_f = 2 * M * C * (3 + (1 if has_res else 0))  # stats read + apply read + write (+ res)
            xr = x.clone().requires_grad_()
            gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
            rr = res.clone().requires_grad_() if has_res else None
            out = BN.bn_act(xr, gr, br, rm, rv, rr, True, 0.1, 1e-5, True)
            dy = torch.randn_like(out)
            t_b = timeit(lambda: torch.autograd.grad(out, [xr], dy, retain_graph=True))
            nbytes_b = 2 * M * C * (2 * 3 + 1 + (1 if has_res else 0))  # stats pass (dy, x, y) + apply pass + dx (+ dres)
            print(f"M {M:7d} C {C:4d} res {int(has_res)}: fwd {t_f:.3f} ms ({nbytes_f / t_f / 1e6:.0f} GB/s incl. stats "
                  f"pass)  bwd {t_b:.3f} ms ({nbytes_b / t_b / 1e6:.0f} GB/s incl. stats pass)", flush=True)
            del y, out


if __name__ == "__main__":
    main()
