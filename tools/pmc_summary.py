"""Summarise a rocprofv3 --pmc run: per kernel, achieved MFMA bf16 TFLOP/s
(SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / kernel time) and MFMA-busy share."""
import collections
import csv
import sys


def main(path, title):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: {"mops": 0.0, "busy": 0.0, "active": 0.0, "ns": 0, "n": 0})
    seen = set()
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        d = per[k]
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        if c == "SQ_INSTS_VALU_MFMA_MOPS_BF16":
            d["mops"] += v
        elif c == "SQ_VALU_MFMA_BUSY_CYCLES":
            d["busy"] += v
        elif c == "GRBM_GUI_ACTIVE":
            d["active"] += v
        key = (r["Dispatch_Id"], k)
        if key not in seen:
            seen.add(key)
            d["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d["n"] += 1
    print(f"# {title}\n\nSource: `{path}` (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE "
          f"SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace).  TFLOP/s = MOPS_BF16 x 512 / dispatch time "
          f"(dense bf16 peak ~2500).\n")
    print("| kernel | dispatches | time ms | MFMA TFLOP/s (bf16) |\n|---|---|---|---|")
    for k, d in sorted(per.items(), key=lambda kv: -kv[1]["ns"])[:20]:
        tf = d["mops"] * 512 / max(d["ns"], 1) / 1e3
        print(f"| `{k}` | {d['n']} | {d['ns'] / 1e6:.2f} | {tf:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "PMC")
