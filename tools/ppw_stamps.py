"""Phase-segment cycle shares of gemm_ppw_kernel (the persistent wave-specialised
GEMM: group 0 issues every LDS-DMA, group 1 every C store) on the BERT-base shapes,
from a stamp build (tools/build_kernel_variant.sh pwN gemm_ppp.hip -DKFA_PW_STAMP=N,
KFA_KERNELS_SO=_hip_kernels_pwN.so).  Segment names and caveats: tools/wgrad_stamps.py.

    KFA_KERNELS_SO=_hip_kernels_pw1.so python tools/ppw_stamps.py 32768x2304x768 ...
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wgrad_stamps import read_stamps, report  # noqa: E402
from kubeflow_controller_amd.ops.gemm import gemm_ppp  # noqa: E402


def run(m: int, n: int, k: int, probe: int) -> None:
    d = torch.device("cuda")
    a = torch.randn(m, k, device=d).to(torch.bfloat16)
    b = torch.randn(n, k, device=d).to(torch.bfloat16)
    for _ in range(20):
        gemm_ppp(a, b, probe=probe, split=False)
    torch.cuda.synchronize()
    report(read_stamps("kfa_pw_stamps"), f"ppw{'-nt' if probe == 10 else ''} {m}x{n}x{k}")


if __name__ == "__main__":
    for arg in sys.argv[1:] or ["32768x2304x768", "32768x3072x768", "32768x768x3072", "32768x768x768"]:
        run(*map(int, arg.split("x")), probe=9)
