"""Static instruction mix of the kernels in a gfx950 assembly file (hipcc -S).

Counts, per kernel, the instructions of each class in the emitted code — not a
dynamic count (loops count once), but for fully unrolled kernels such as the
S = 128 attention it is the per-wave issue count, and it moves one-for-one with
SQ_INSTS_VALU.  Transcendentals (exp / log / rcp / sqrt) are quarter rate and
listed separately.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -o a.s csrc/kernels/attention.hip
    python tools/isa_mix.py a.s [name-substring]
"""
import re
import sys
from collections import Counter

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def classify(op: str) -> str:
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait/barrier/nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main() -> int:
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    kern, counts, ops = None, {}, {}
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and "@" not in m.group(1):
            name = m.group(1)
            if name.startswith("_Z") or "kernel" in name:
                kern = name
                counts.setdefault(kern, Counter())
                ops.setdefault(kern, Counter())
            continue
        if line.startswith("\t.end_amdhsa_kernel") or line.startswith(".Lfunc_end"):
            kern = None if line.startswith(".Lfunc_end") else kern
            continue
        if kern is None:
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        if not re.match(r"^[a-z_0-9]+$", op):
            continue
        counts[kern][classify(op)] += 1
        ops[kern][op] += 1
    for k, c in counts.items():
        if filt and filt not in k:
            continue
        tot = sum(c.values())
        print(f"{k}: total {tot}  " + "  ".join(f"{n}={c[n]}" for n in
                                                  ("valu", "trans", "mfma", "salu", "lds", "vmem", "wait/barrier/nop")))
        if filt:
            for op, n in ops[k].most_common(40):
                print(f"    {op:32s} {n}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
