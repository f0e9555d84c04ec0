"""Where wgrad_pp_kernel's k-loop spends its cycles: run a weight-gradient shape
on a stamp build (tools/build_kernel_variant.sh stN wgrad.hip -DKFA_WP_STAMP=N,
selected with KFA_KERNELS_SO=_hip_kernels_stN.so) and print, per wave group, the
share of each segment of the four phases of a k-tile:

    issue   ds_reads + this phase's LDS-DMA issue           (stamp build 2 only)
    vmcnt   the counted DMA retire                          (stamp build 2 only)
    bar1    s_barrier + lgkmcnt(0) before the MFMAs         (build 1: issue+vmcnt+bar1)
    mfma    the 16 MFMAs of the phase
    bar2    the s_barrier after them

plus the prologue and the epilogue (partial-tile stores drained).  Shares, not
run times: every stamp drains LDS reads in flight (cdna_hip_programming.md §7).

    KFA_KERNELS_SO=_hip_kernels_st1.so python tools/wgrad_stamps.py 32768x2304x768 ...
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_controller_amd.ops import _lib  # noqa: E402
from kubeflow_controller_amd.ops.conv import wgrad_into  # noqa: E402

SEG = 24
NAMES = ["bar1", "mfma", "bar2", "issue", "vmcnt"]


def run(rows: int, co: int, ci: int) -> None:
    d = torch.device("cuda")
    x = torch.randn(rows, ci, device=d).to(torch.bfloat16)
    dy = torch.randn(rows, co, device=d).to(torch.bfloat16)
    out = torch.zeros(co, ci, device=d)
    for _ in range(20):
        wgrad_into(x, dy, out, 1, 1, rows, ci, 1, rows, co, 1, 1, 1, 0, accumulate=True)
    torch.cuda.synchronize()
    report(read_stamps("kfa_wp_stamps"), f"{rows}x{co}x{ci}")


def read_stamps(sym: str) -> np.ndarray:
    buf = np.zeros(256 * 2 * SEG, dtype=np.uint32)
    fn = getattr(_lib.lib(), sym)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rc = fn(buf.ctypes.data, buf.size)
    assert rc == 0, rc
    return buf


def report(buf: np.ndarray, label: str) -> None:
    """Per wave group: shares of prologue / k-loop / epilogue and the mean cycles
    of each phase segment per k-tile (blocks whose stamp record is non-empty)."""
    s = buf.reshape(256, 2, SEG).astype(np.float64)
    live = s[:, 0, 22] > 0
    s = s[live]
    print(f"{label}: {live.sum()} blocks, {s[:, 0, 22].mean():.0f} k-tiles per block")
    for grp in range(2):
        g = s[:, grp, :].mean(axis=0)
        loop = g[:20].sum()
        tot = loop + g[20] + g[21]
        kt = s[:, grp, 22].mean()
        print(f"  group {grp}: {tot:,.0f} cycles per block; prologue {g[20] / tot:5.1%}, "
              f"k-loop {loop / tot:5.1%} ({loop / kt:,.0f} cycles per k-tile), epilogue {g[21] / tot:5.1%}")
        for ph in range(4):
            cells = []
            for k in (3, 4, 0, 1, 2):
                if ph == 3 and k == 4 and not (g[3] > 0):  # stamp build 3: slot 19 = k-tile entry
                    continue
                v = g[ph * 5 + k]
                if v > 0:
                    cells.append(f"{NAMES[k]} {v / kt:6.0f}")
            print(f"    phase {ph}: " + "  ".join(cells) + "   (cycles per k-tile)")
        if g[19] > 0 and not g[3] > 0:
            print(f"    k-tile entry (tail of the previous k-tile: advance, loop branch): {g[19] / kt:6.0f}")


if __name__ == "__main__":
    for a in sys.argv[1:] or ["32768x2304x768", "32768x768x3072", "32768x768x768"]:
        run(*map(int, a.split("x")))
