"""Where a kernel sits in a rocprofv3 kernel trace: for every launch of the kernels
whose name contains NEEDLE, its duration and the kernels launched just before and
after it on the same queue (the code path that issues it).

    python tools/trace_context.py trace.csv __amd_rocclr_copyBuffer [max_rows]
"""
import collections
import csv
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]


def main() -> int:
    path, needle = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    q = collections.defaultdict(list)
    for r in rows:
        q[r.get("Queue_Id", "0")].append(r)
    ctx = collections.Counter()
    durs = []
    for lst in q.values():
        for i, r in enumerate(lst):
            if needle in r["Kernel_Name"]:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                durs.append(d)
                before = short(lst[i - 1]["Kernel_Name"]) if i else "-"
                after = short(lst[i + 1]["Kernel_Name"]) if i + 1 < len(lst) else "-"
                ctx[(before, after)] += 1
    print(f"{len(durs)} launches, mean {sum(durs) / max(1, len(durs)):.2f} us, total {sum(durs):.1f} us")
    for (b, a), n in ctx.most_common(lim):
        print(f"{n:5d}  after {b}  |  before {a}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
