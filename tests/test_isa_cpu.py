"""ISA checks of the hand-scheduled kernels (CPU: hipcc cross-compiles gfx950).

The ping-pong weight gradient and the lockstep wgrad read their MFMA operands
with inline-asm `ds_read_b64_tr_b16` (`csrc/kernels/wgrad.hip`, `ds_tr16`): hipcc
would otherwise wait `vmcnt(0)` for the LDS-DMAs in flight before every phase's
reads.  Inline asm moves two duties to the kernel: every read must be waited for
by the kernel's own `lgkmcnt` before its registers are used, and hipcc must not
place an instruction that touches a still-loading register in between — checked
here on the compiled `.s` with tools/asm_read_hazards.py — and the compiler's
drain must really be gone from the loops.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HIPCC = os.environ.get("HIPCC") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc"))
pytestmark = pytest.mark.skipif(not HIPCC, reason="hipcc not available")


@pytest.fixture(scope="module")
def wgrad_s(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "wgrad.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    f"-I{ROOT}/csrc/kernels", "--cuda-device-only", "-S", f"{ROOT}/csrc/kernels/wgrad.hip",
                    "-o", str(out)], check=True, capture_output=True, timeout=600)
    return out.read_text()


def _bodies(text: str, pat: str):
    for name in re.findall(r"^(_Z[^:\s]+):", text, re.M):
        if pat in name:
            i = text.index(name + ":")
            yield name, text[i:text.index(".Lfunc_end", i)].split("\n")


def _meta(text: str, name: str, key: str) -> int:
    seg = text[text.rindex("- .agpr_count", 0, text.index(".name:           " + name)):]
    return int(re.search(rf"\.{key}:\s+(\d+)", seg).group(1))


def test_asm_operand_reads_have_no_hazards(wgrad_s):
    import asm_read_hazards
    found = 0
    for name, body in _bodies(wgrad_s, "wgrad"):
        if not any("ds_read_b64_tr_b16" in l for l in body):
            continue
        found += 1
        assert asm_read_hazards.check(body) == [], name
    assert found >= 7  # wgrad_pp_kernel<false / true> + six lockstep variants


def test_no_compiler_vmcnt_before_operand_reads_in_pp_loop(wgrad_s):
    for name, body in _bodies(wgrad_s, "wgrad_pp_kernel"):
        labels = {m.group(1): k for k, l in enumerate(body) if (m := re.match(r"^\.(LBB\d+_\d+):", l))}
        loops = [(labels[m.group(1)], k) for k, l in enumerate(body)
                 if (m := re.search(r"s_c?branch\w* \.(LBB\d+_\d+)", l)) and m.group(1) in labels
                 and labels[m.group(1)] < k]
        main = max(loops, key=lambda x: x[1] - x[0])
        waits = [k for k in range(*main) if re.match(r"\s+s_waitcnt vmcnt", body[k])
                 and "ASM" not in body[k - 1] and any("ds_read" in x for x in body[k + 1:k + 4])]
        assert waits == [], (name, waits)


def test_pp_kernels_do_not_spill_in_the_loop(wgrad_s):
    for name, _ in _bodies(wgrad_s, "wgrad_pp_kernel"):
        assert _meta(wgrad_s, name, "vgpr_count") <= 256
        # the pointwise variant parks two values across its k-loop (4 scratch ops per wave in total)
        assert _meta(wgrad_s, name, "vgpr_spill_count") <= 2, name


@pytest.fixture(scope="module")
def conv_s(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "conv_igemm.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    f"-I{ROOT}/csrc/kernels", "--cuda-device-only", "-S", f"{ROOT}/csrc/kernels/conv_igemm.hip",
                    "-o", str(out)], check=True, capture_output=True, timeout=900)
    return out.read_text()


def test_conv_asm_fragment_reads_have_no_hazards(conv_s):
    """conv_igemm_kernel's 4-wave tiles (and the BatchNorm-prologue forms) read their
    MFMA fragments with inline-asm ds_read_b128 and counted lgkmcnt waits
    (csrc/kernels/conv_igemm.hip, `compute`)."""
    import asm_read_hazards
    found = 0
    for name, body in _bodies(conv_s, "conv_igemm_kernel"):
        if not any(l.strip() == ";;#ASMSTART" and "ds_read" in nxt for l, nxt in zip(body, body[1:])):
            continue
        found += 1
        assert asm_read_hazards.check(body) == [], name
    assert found >= 32  # 128x128, 128x64, 256x64 x 8 epilogues + the 8 prologue forms


def test_conv_kernels_do_not_spill(conv_s):
    for name, _ in _bodies(conv_s, "conv_"):
        if "Lj31E" in name:  # kEpiAll (pick_epi's catch-all, the ReLU mask read from y): off the ResNet step
            continue
        assert _meta(conv_s, name, "vgpr_spill_count") == 0, name
