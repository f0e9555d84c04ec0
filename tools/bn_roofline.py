"""Effective bandwidth of the ResNet-50 BatchNorm passes from a kernel-trace summary.

HBM counters (FETCH_SIZE / WRITE_SIZE) miss the Infinity-Cache hits, so they
understate what a streaming pass moves.  This tool counts the bytes each BN
kernel class MUST move from the tensor shapes of ResNet-50 v1.5 at batch N and
224x224 (bf16 activations, 1-bit ReLU masks) and divides by the measured time
per step from a ``tools/profile_summary.py`` table:

    python tools/bn_roofline.py profiles/r3_resnet50_bs256_head.md [N]

Kernel classes (csrc/kernels/batchnorm.hip; calls per step in brackets):
  bn_apply<true,false,false,false>   bn1/bn2 forward                 x -> y          4 B/el
  bn_apply<true,true,true,false>     identity-block bn3 (+res, bits)  x,res -> y,bits 6.125
  bn_apply<true,true,true,true>      downsample-block bn3 + bn_ds     x,r -> y,bits   6.125
  bn_bwd_apply<2,false>              bn1/bn2 (+stem) backward         dy,x -> dx      6
  bn_bwd_apply<3,false>              identity bn3 + bn_ds backward    dy,x,bits -> dx 6.125
  bn_bwd_apply_rstats<3>             downsample-block bn3 backward    dy,x,r,bits->dx 8.125
"""
import re
import sys

STAGES = [(3, 64, 56), (4, 128, 28), (6, 256, 14), (3, 512, 7)]


def elements(N=256):
    e = {k: 0 for k in ("bn12", "bn3_id", "bn3_ds", "stem")}
    s_in = 56
    for si, (blocks, mid, s) in enumerate(STAGES):
        for b in range(blocks):
            sp_in = s_in if b == 0 else s
            e["bn12"] += N * sp_in * sp_in * mid + N * s * s * mid      # bn1 (at the conv1 input res), bn2
            if b == 0:
                e["bn3_ds"] += N * s * s * 4 * mid                        # bn3 == bn_ds size
            else:
                e["bn3_id"] += N * s * s * 4 * mid
        s_in = s
    e["stem"] = N * 112 * 112 * 64
    return e


def main():
    md = open(sys.argv[1]).read()
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    ms = {m.group(1): float(m.group(2)) for m in re.finditer(r"\| `([^`]+)` \| [^|]+ \| ([0-9.]+) \|", md)}
    e = elements(N)
    rows = [
        ("bn_apply<true, false, false, false>", e["bn12"] * 4),
        ("bn_apply<true, true, true, false>", e["bn3_id"] * 6.125),
        ("bn_apply<true, true, true, true>", e["bn3_ds"] * 6.125),
        ("bn_bwd_apply<2, false>", (e["bn12"] + e["stem"]) * 6),
        ("bn_bwd_apply<3, false>", (e["bn3_id"] + e["bn3_ds"]) * 6.125),
        ("bn_bwd_apply_rstats<3>", e["bn3_ds"] * 8.125),
    ]
    print("| kernel | GB moved / step | ms / step | effective TB/s | % of 6.3 TB/s (measured copy peak) |")
    print("|---|---:|---:|---:|---:|")
    tot_b = tot_t = 0.0
    for k, b in rows:
        t = next((v for n, v in ms.items() if n.replace(" ", "").startswith(k.replace(" ", ""))), None)
        if t is None:
            continue
        tot_b += b
        tot_t += t
        print(f"| `{k}` | {b / 1e9:.2f} | {t:.3f} | {b / t / 1e9:.2f} | {100 * b / t / 1e9 / 6.3:.0f} % |")
    print(f"| all apply passes | {tot_b / 1e9:.2f} | {tot_t:.3f} | {tot_b / tot_t / 1e9:.2f} | "
          f"{100 * tot_b / tot_t / 1e9 / 6.3:.0f} % |")


if __name__ == "__main__":
    main()
