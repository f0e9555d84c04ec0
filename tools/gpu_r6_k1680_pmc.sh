#!/bin/bash
# PMC passes over the W&D layer-1 GEMM: own fwd vs own on the dgrad shape vs hipBLASLt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6k1680; mkdir -p $O
export TMPDIR=/tmp KFA_PMC_MODE=1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY \
  --kernel-include-regex 'gemm_pp|Cijk' --output-format csv -d $O/p1 -o p -- python -u tools/bench_wd_k1680.py > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
  --kernel-include-regex 'gemm_pp|Cijk' --output-format csv -d $O/p2 -o p -- python -u tools/bench_wd_k1680.py > $O/p2.log 2>&1 || exit 1
