#!/usr/bin/env python3
"""Markdown per-shape roofline table of the conv launches in a
``tools/launch_profile.py`` output: for every (fwd/dgrad, M, N, K, taps, addend,
tile variant) the per-step time, the MFMA and HBM floors (2.0 PFLOP/s bf16 dense
at the clock the chip holds under load; 6.0 TB/s, a float4 copy's rate) and what
the launch reaches.

    python tools/launch_rooflines.py gpurun_out/r6lp/r50_launches.txt > profiles/x.md
"""
import collections
import re
import sys

PF, TBS = 2.0e15, 6.0e12


def main():
    path = sys.argv[1]
    agg = collections.defaultdict(list)
    wg = collections.defaultdict(list)
    for l in open(path):
        m = re.match(r"\s*(\d+) (kfa_conv_\S+)\s+([\d.]+) us\s+\((.*)\)", l)
        if not m:
            continue
        name, us, a = m.group(2), float(m.group(3)), [int(x) for x in m.group(4).split(",")]
        if name == "kfa_conv_igemm":
            Nb, H, W, C, P, Q, R, S, sa, ra = a[:10]
            N, var, E = a[18], a[19], a[20]
            agg[("dgrad" if ra < 0 else "fwd", Nb * P * Q, N, R * S * C, R, E, var, Nb * H * W * C)].append(us)
        elif name == "kfa_conv_igemm_bnpro":
            Nb, H, W, C, P, Q, R, S, st, pad, N, var = a[:12]
            agg[("fwd+bn", Nb * P * Q, N, R * S * C, R, 0, var, Nb * H * W * C)].append(us)
        elif name == "kfa_conv_wgrad":
            _, _, Nb, H, W, Ci, P, Q, Co, R, S, st = a[:12]
            wg[(Co, Ci, R, st, Nb * P * Q, Nb * H * W * Ci)].append(us)
    print("| conv launch | calls | us / call | MFMA floor | HBM floor | TF/s | TB/s | gap us / step |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    rows, tot, tfl = [], 0.0, 0.0
    for (kind, M, N, K, R, E, var, tin), v in agg.items():
        t = sum(v) / len(v)
        fl = 2.0 * M * N * K
        by = tin * 2 + M * N * 2 * (1 + (2 if E else 0)) + N * K * 2
        f_m, f_b = fl / PF * 1e6, by / TBS * 1e6
        floor = max(f_m, f_b)
        tot += sum(v)
        tfl += floor * len(v)
        rows.append(((t - floor) * len(v), f"| {kind} M={M} N={N} K={K} {R}x{R}{' +E' if E else ''} v{var} | {len(v)} | "
                     f"{t:.1f} | {f_m:.1f} | {f_b:.1f} | {fl / t / 1e6:.0f} | {by / t / 1e6:.2f} | {(t - floor) * len(v):.0f} |"))
    for _, r in sorted(rows, reverse=True):
        print(r)
    print(f"\nimplicit-GEMM conv (fwd + dgrad): {tot / 1e3:.2f} ms / step measured vs {tfl / 1e3:.2f} ms of floors\n")
    print("| weight gradient | calls | us / call | MFMA floor | HBM floor (inputs only) | TF/s |")
    print("|---|---:|---:|---:|---:|---:|")
    rows, tot, tfl = [], 0.0, 0.0
    for (Co, Ci, R, st, M, tin), v in wg.items():
        t = sum(v) / len(v)
        fl = 2.0 * M * Co * R * R * Ci
        by = M * Co * 2 + tin * 2
        f_m, f_b = fl / PF * 1e6, by / TBS * 1e6
        tot += sum(v)
        tfl += max(f_m, f_b) * len(v)
        rows.append(((t - max(f_m, f_b)) * len(v), f"| dW {Co}x{R}x{R}x{Ci} s{st} over {M} px | {len(v)} | {t:.1f} | "
                     f"{f_m:.1f} | {f_b:.1f} | {fl / t / 1e6:.0f} |"))
    for _, r in sorted(rows, reverse=True):
        print(r)
    print(f"\nweight gradients (incl. the split-K reduce launches): {tot / 1e3:.2f} ms / step vs {tfl / 1e3:.2f} ms of floors")


if __name__ == "__main__":
    main()
