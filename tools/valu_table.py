"""Per-kernel issue mix from one rocprofv3 --pmc pass (tools/gpu_valu_pmc.sh):

    python tools/valu_table.py gpurun_out/valu/r50/p_counter_collection.csv

VALU busy = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) — the share
of SIMD cycles spent issuing vector ALU work (SQ counts in quad-cycles; GRBM sums the
8 XCDs).  A kernel near 100 % is VALU-bound; MFMA / VALU shows how much scalar-vector
work rides on each matrix instruction.  Rows sorted by total time.
"""
import collections
import csv
import sys


def main(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:52]
        d = r["Dispatch_Id"]
        per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[(k, d)] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for (k, d), cs in per.items():
        for c, v in cs.items():
            agg[k][c] += v
        agg[k]["_ns"] += dur[(k, d)]
        n[k] += 1
    print("| kernel | calls | mean us | VALU busy | VALU / wave | SALU / wave | MFMA / wave | LDS / wave | VALU per MFMA |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k, m in sorted(agg.items(), key=lambda kv: -kv[1]["_ns"]):
        w = m.get("SQ_WAVES", 0) or 1
        g = m.get("GRBM_GUI_ACTIVE", 0)
        busy = m.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (g / 8 * 1024) if g else 0
        mf = m.get("SQ_INSTS_MFMA", 0)
        print(f"| `{k}` | {n[k]} | {m['_ns'] / n[k] / 1e3:.1f} | {100 * busy:.0f}% | {m.get('SQ_INSTS_VALU', 0) / w:.0f} | "
              f"{m.get('SQ_INSTS_SALU', 0) / w:.0f} | {mf / w:.0f} | {m.get('SQ_INSTS_LDS', 0) / w:.0f} | "
              f"{(m.get('SQ_INSTS_VALU', 0) / mf) if mf else float('nan'):.1f} |")


if __name__ == "__main__":
    main(sys.argv[1])
