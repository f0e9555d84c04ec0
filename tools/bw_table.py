"""Achieved HBM bandwidth per kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, kB per dispatch) over the same workload.

    python tools/bw_table.py <fetch counter_collection.csv> <write counter_collection.csv>

Per kernel name: dispatches, mean duration (profiled, so a little slower than an
unprofiled run), mean MB fetched / written, (fetch + write) / duration in TB/s,
and that as a share of the ≈8 TB/s HBM3E peak.  Sorted by total time.
"""
import collections
import csv
import sys

PEAK_TBS = 8.0


def load(path, counter):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        d = r["Dispatch_Id"]
        per[k][d] += float(r["Counter_Value"])
        dur[k][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, dur


def main(fetch_csv, write_csv):
    f, fd = load(fetch_csv, "FETCH_SIZE")
    w, wd = load(write_csv, "WRITE_SIZE")
    rows = []
    for k in f:
        if k not in w:
            continue
        n = len(f[k])
        t_ns = (sum(fd[k].values()) / n + sum(wd[k].values()) / len(wd[k])) / 2
        mb_f = sum(f[k].values()) / n / 1e3
        mb_w = sum(w[k].values()) / len(w[k]) / 1e3
        tbs = (mb_f + mb_w) * 1e6 / t_ns / 1e3 if t_ns else 0.0
        rows.append((t_ns * n, k, n, t_ns, mb_f, mb_w, tbs))
    rows.sort(reverse=True)
    print("| kernel | dispatches | mean us | MB fetched | MB written | TB/s | % of 8 TB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for _, k, n, t, mf, mw, tbs in rows:
        print(f"| `{k}` | {n} | {t / 1e3:.1f} | {mf:.1f} | {mw:.1f} | {tbs:.2f} | {100 * tbs / PEAK_TBS:.0f} |")


if __name__ == "__main__":
    main(*sys.argv[1:3])
