"""Scan gfx950 device assembly for a VMEM store of more than 64 bits of data
(dwordx3 / dwordx4) whose data VGPRs a VALU op overwrites before two wait states
have passed (the rule: cdna_hip_programming.md §5.7 — such a store ends with
`s_nop 1` in inline asm).

hipcc's hazard pass inserts those wait states inside a basic block but missed
them across a branch join inside a loop (conv_igemm_kernel's PRO side store:
the next chunk's first VALU op overwrote the store's 2nd data dword on some
lanes, docs/kernels.md).  Usage:

    python tools/asm_hazard_scan.py csrc/kernels/conv_igemm.hip [more.hip ...]

Exit status 1 if any site is found (each printed with its kernel and the
offending instruction).
"""
import os
import re
import subprocess
import sys
import tempfile

_STORE = re.compile(r"(buffer|global|flat)_store_dwordx(3|4)$")  # data wider than 64 bits


def _regs(tok: str) -> set:
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan_asm(text: str, need: int = 2):
    """[(line, kernel, store, overwriting instruction, wait states)] of hazard sites."""
    out, func = [], None
    lines = text.split("\n")
    for i, line in enumerate(lines):
        if re.match(r"^_Z\S*:", line):
            func = line[:-1]
        t = line.strip()
        parts = t.replace(",", " ").split()
        if not parts or not _STORE.match(parts[0]):
            continue
        data = parts[2] if parts[0].startswith(("global", "flat")) else parts[1]
        dregs, ws = _regs(data), 0
        for u in lines[i + 1:i + 16]:
            u = u.strip()
            if not u or u.startswith((";", ".")) or u.endswith(":"):
                continue
            p = u.replace(",", " ").split()
            if p[0] in ("s_endpgm", "s_branch", "s_setpc_b64"):  # the next line is not the next instruction
                break
            if p[0] == "s_nop":
                ws += int(p[1], 0) + 1
            else:
                if p[0].startswith("v_") and len(p) > 1 and _regs(p[1]) & dregs and ws < need:
                    out.append((i + 1, func, t, u, ws))
                    break
                ws += 1
            if ws >= need:
                break
    return out


def compile_asm(src: str) -> str:
    inc = os.path.dirname(os.path.abspath(src))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", inc, "--cuda-device-only", "-S",
                        src, "-o", out], check=True, capture_output=True)
        return open(out).read()


def main(srcs) -> int:
    bad = 0
    for src in srcs:
        hits = scan_asm(compile_asm(src))
        for line, func, st, ov, ws in hits:
            print(f"{src}: asm line {line} {func}\n    {st}\n    -> {ov} ({ws} wait states)")
        bad += len(hits)
        print(f"{src}: {len(hits)} store-data hazard site(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
