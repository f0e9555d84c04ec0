"""Device-assembly check (CPU, hipcc cross-compile): no VMEM store's data VGPRs
are overwritten before the required wait states (tools/asm_hazard_scan.py)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_scanner_flags_the_pattern():
    import asm_hazard_scan as h
    asm = "\n".join(["_Zk:", "\tbuffer_store_dwordx4 v[98:101], v122, s[48:51], s63 offen", ".LBB0_2:",
                     "\tv_lshlrev_b32_e32 v99, 16, v10"])
    assert len(h.scan_asm(asm)) == 1
    ok = asm.replace(".LBB0_2:", ".LBB0_2:\n\ts_nop 1")
    assert h.scan_asm(ok) == []


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
@pytest.mark.timeout(600)
def test_conv_igemm_has_no_store_data_hazard():
    import asm_hazard_scan as h
    src = os.path.join(ROOT, "csrc", "kernels", "conv_igemm.hip")
    assert h.scan_asm(h.compile_asm(src)) == []
