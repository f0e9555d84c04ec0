"""Check a kernel's .s for uses of registers still being filled by an inline-asm
LDS read.  hipcc treats an asm output as written when the asm statement ends, so
a compiler-placed instruction (a copy, an address reuse, an MFMA hoisted above the
wait) that touches such a register before the kernel's own `s_waitcnt lgkmcnt(0)`
would see stale data.  Every asm `ds_read*` destination stays "in flight" until
the next wait that retires it: lgkmcnt(0), or a counted lgkmcnt(N) once N younger reads
are outstanding (counting only the asm reads: conservative); any other
instruction that names one of those registers — including as the address of a
later read — is reported.

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/kernels/wgrad.hip -o /tmp/wgrad.s
    python tools/asm_read_hazards.py /tmp/wgrad.s wgrad_pp_kernel
"""
import re
import sys


def regs_of(line: str) -> set:
    out = set()
    for a, b in re.findall(r"v\[(\d+):(\d+)\]", line):
        out |= set(range(int(a), int(b) + 1))
    out |= {int(a) for a in re.findall(r"\bv(\d+)\b", line)}
    return out


def check(body: list) -> list:
    pending, bad, in_asm = [], [], False  # in issue order: the register sets of asm reads in flight
    for k, line in enumerate(body):
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        w = re.search(r"lgkmcnt\((\d+)\)", t)
        if w:
            n = int(w.group(1))
            pending = pending[len(pending) - n:] if n else []
            continue
        live = set().union(*pending) if pending else set()
        m = re.match(r"ds_read\w*\s+(v\[\d+:\d+\]|v\d+),\s*(v\d+)", t)
        if m and in_asm:
            if int(m.group(2)[1:]) in live:
                bad.append((k, t))
            pending.append(regs_of(m.group(1)))
            continue
        if live and re.match(r"[vsb]\w*_|ds_|buffer_|global_", t) and regs_of(t) & live:
            bad.append((k, t))
    return bad


def main() -> int:
    path, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read()
    names = [n for n in re.findall(r"^(_Z[^:\s]+):", text, re.M) if pat in n]
    total = 0
    for n in names:
        i = text.index(n + ":")
        body = text[i:text.index(".Lfunc_end", i)].split("\n")
        bad = check(body)
        total += len(bad)
        print(f"{len(bad):4d}  {n[:100]}")
        for k, t in bad[:8]:
            print(f"        line {k}: {t}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
