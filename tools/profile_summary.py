"""Turn a rocprofv3 ``--kernel-trace`` CSV into a committed markdown summary.

    python tools/profile_summary.py gpurun_out/prof/r50_kernel_trace.csv STEPS STEP_MS "title" > profiles/x.md

Only the last ``STEPS`` steps' worth of kernels (by wall window) are counted, so
warm-up / autotuning launches do not pollute the per-step numbers.  Kernels
are grouped into own HIP kernels (``kfa``'s anonymous-namespace kernels) vs
vendor libraries (hipBLASLt ``Cijk_*``, MIOpen / CK) vs PyTorch elementwise.
"""
import collections
import csv
import sys

OWN_MARKERS = ("(anonymous namespace)::", "kfa_radix::")
LIB_MARKERS = ("at::", "c10::", "rocprim::", "hipcub::", "cub::")
ANCHOR = "sgd_kernel"  # one launch per training step (fused SGD over the flat parameter group)


def origin(name: str) -> str:
    # library namespaces first: ATen's own anonymous-namespace kernels (e.g.
    # at::native::(anonymous namespace)::indexFuncLargeIndex) are not ours
    if name.startswith("Cijk_") or name.startswith("Custom_Cijk"):
        return "hipBLASLt"
    if "rocprim::" in name or "hipcub::" in name or "cub::" in name:
        return "rocPRIM / hipCUB"
    if any(m in name for m in LIB_MARKERS):
        return "PyTorch ATen"
    if any(m in name for m in OWN_MARKERS):
        return "own HIP (csrc/kernels)"
    if "igemm_" in name or "ck::" in name or name.startswith("_ZN2ck") or "SubTensor" in name or "MIOpen" in name:
        return "MIOpen / CK"
    if "at::native" in name:
        return "PyTorch ATen"
    if "rocclr" in name:
        return "runtime copy / fill"
    return "other"


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:90]


def main(path, steps, step_ms, title):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # Anchor on the once-per-step optimizer kernel when present: the window is then exactly
    # the last STEPS steps (from the end of one optimizer launch to the end of the last).
    anchors = []
    for i, r in enumerate(rows):  # one optimizer launch per flat group: adjacent launches = one step
        if ANCHOR in r["Kernel_Name"]:
            if anchors and i - anchors[-1] <= 3:
                anchors[-1] = i
            else:
                anchors.append(i)
    if len(anchors) > steps:
        win = rows[anchors[-steps - 1] + 1:anchors[-1] + 1]
        step_ms = (int(win[-1]["End_Timestamp"]) - int(rows[anchors[-steps - 1]]["End_Timestamp"])) / 1e6 / steps
    else:
        end = int(rows[-1]["End_Timestamp"])
        win = [r for r in rows if int(r["Start_Timestamp"]) > end - steps * step_ms * 1e6]
    per = collections.defaultdict(lambda: [0, 0])
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[r["Kernel_Name"]][0] += d
        per[r["Kernel_Name"]][1] += 1
    tot = sum(v[0] for v in per.values())
    by_origin = collections.defaultdict(float)
    for k, (d, _) in per.items():
        by_origin[origin(k)] += d
    print(f"# {title}\n")
    print(f"Source: `{path}` (rocprofv3 --kernel-trace --stats), last {steps} steps "
          f"(window {steps * step_ms:.1f} ms).\n")
    # wall-clock union of the kernel intervals: kernels on a side stream that overlap
    # the main stream's are counted once (the sum above counts both)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win)
    union, cur_s, cur_e = 0, None, None
    for a, b in iv:
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        union += cur_e - cur_s
    print(f"Kernel-busy time per step: **{tot / steps / 1e6:.2f} ms** summed over kernels, "
          f"{union / steps / 1e6:.2f} ms GPU-busy wall clock (overlapping streams counted once) "
          f"({len(win) / steps:.0f} launches/step)\n")
    print("| origin | ms/step | share |\n|---|---|---|")
    for k, v in sorted(by_origin.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {v / steps / 1e6:.2f} | {100 * v / tot:.1f}% |")
    print("\n| kernel | origin | ms/step | calls/step |\n|---|---|---|---|")
    for k, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:30]:
        print(f"| `{short(k)}` | {origin(k)} | {d / steps / 1e6:.3f} | {c / steps:.1f} |")


if __name__ == "__main__":
    if len(sys.argv) > 5:
        ANCHOR = sys.argv[5]
    main(sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else "profile")
