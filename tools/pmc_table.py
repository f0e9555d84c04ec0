"""Per-kernel table of rocprofv3 --pmc counters (mean per dispatch) from one or
more ``*_counter_collection.csv`` files.

    python tools/pmc_table.py gpurun_out/pmc1/x_counter_collection.csv gpurun_out/pmc2/x_counter_collection.csv
"""
import collections
import csv
import sys


def main(paths):
    # counter -> {dispatch: summed value}; a counter's mean is over the dispatches of ITS pass
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    ns = collections.defaultdict(dict)
    for path in paths:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            if r.get("Grid_Size"):
                k += f" [grid {r['Grid_Size']}]"
            d = (path, r["Dispatch_Id"])
            vals[k][r["Counter_Name"]][d] += float(r["Counter_Value"])
            ns[k][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, cs in vals.items():
        t = sum(ns[k].values()) / max(len(ns[k]), 1)
        print(f"## {k}  (mean dispatch {t / 1e3:.1f} us over {len(ns[k])} dispatches)")
        for c, per_d in sorted(cs.items()):
            print(f"  {c:36s} {sum(per_d.values()) / len(per_d):16.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])
