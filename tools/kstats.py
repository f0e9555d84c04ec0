"""Summarise a rocprofv3 kernel trace: per-kernel ms/step over the last N steps."""
import collections
import csv
import sys


def main(path, steps, step_ms, top=40):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    end = int(rows[-1]["End_Timestamp"])
    win = [r for r in rows if int(r["Start_Timestamp"]) > end - steps * step_ms * 1e6]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"][:110]][0] += d
        agg[r["Kernel_Name"][:110]][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"kernels in window: {len(win)}  busy ms/step: {tot / steps / 1e6:.2f}")
    cat = collections.defaultdict(float)
    for k, (d, c) in agg.items():
        n = k.lower()
        if "bn_" in n or "batch_norm" in n:
            c_ = "batchnorm"
        elif "conv" in n or "igemm" in n or "gemm" in n or k.startswith("Cijk"):
            c_ = "conv/gemm"
        elif "elementwise" in n:
            c_ = "elementwise"
        else:
            c_ = "other"
        cat[c_] += d / steps / 1e6
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"  {k:14s} {v:8.2f} ms/step")
    for k, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{d / steps / 1e6:8.3f} ms {c / steps:6.1f}/step  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 40)
