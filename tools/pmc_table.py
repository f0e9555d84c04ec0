"""Per-kernel table of rocprofv3 --pmc counters (mean per dispatch) from one or
more ``*_counter_collection.csv`` files.

    python tools/pmc_table.py gpurun_out/pmc1/x_counter_collection.csv gpurun_out/pmc2/x_counter_collection.csv
"""
import collections
import csv
import sys


def main(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    ns = collections.defaultdict(dict)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            ns[k][(path, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, cs in vals.items():
        t = sum(ns[k].values()) / max(len(ns[k]), 1)
        print(f"## {k}  (mean dispatch {t / 1e3:.1f} us over {len(ns[k])} dispatches)")
        for c, v in sorted(cs.items()):
            per = sum(v) / max(len(ns[k]), 1)
            print(f"  {c:36s} {per:16.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])
