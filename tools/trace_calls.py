#!/usr/bin/env python3
"""Per-call durations of selected kernels over the last N steps of a rocprofv3 kernel
trace, by position within the step (the i-th launch of the kernel in a step):

    python tools/trace_calls.py trace.csv STEPS ANCHOR_SUBSTR KERNEL_SUBSTR [KERNEL_SUBSTR ...]

Steps are cut at each launch of ANCHOR_SUBSTR (one per step, e.g. the optimizer);
prints the mean duration (us) per position of each kernel pattern, plus the
total per step."""
import collections
import csv
import sys


def main():
    path, steps, anchor = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    pats = sys.argv[4:]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    cuts = [i for i, r in enumerate(rows) if anchor in r[2]]
    cuts = cuts[-(steps + 1):]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for a, b in zip(cuts, cuts[1:]):
        seen = collections.Counter()
        for s, e, n in rows[a + 1:b + 1]:
            for p in pats:
                if p in n:
                    per[p][seen[p]].append((e - s) / 1e3)
                    seen[p] += 1
    for p in pats:
        tot = sum(sum(v) for v in per[p].values()) / max(1, len(cuts) - 1)
        print(f"== {p}: {len(per[p])} launches/step, {tot:.1f} us/step")
        line = []
        for i in sorted(per[p]):
            v = per[p][i]
            line.append(f"{i}:{sum(v) / len(v):.1f}")
        print("  " + " ".join(line))


if __name__ == "__main__":
    main()
