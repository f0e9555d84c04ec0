"""Kernel list of a rocprofv3 kernel trace: every distinct kernel name with its
launches per step (the last ``steps`` steps' window is not needed: counts are
divided by the number of steps the run timed plus warm-up, so compare lists of
runs with the same --steps / --warmup).

    python tools/kernel_list.py trace.csv STEPS > list.txt
    diff <(python tools/kernel_list.py a.csv 8) <(python tools/kernel_list.py b.csv 8)

Used to show that two boxes run identical kernels for one configuration
(routing table ``ops/routes_<arch>.json``: VERDICT r4 "reproducible routing").
"""
import collections
import csv
import sys


def main() -> int:
    path, steps = sys.argv[1], int(sys.argv[2])
    cnt = collections.Counter()
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("kernel_name") or ""
        name = name.replace("(anonymous namespace)::", "").replace("void ", "")
        cnt[name.split("(")[0][:160]] += 1
    for name, n in sorted(cnt.items()):
        print(f"{n / steps:8.2f}  {name}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
