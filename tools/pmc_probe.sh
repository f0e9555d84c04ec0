#!/bin/bash
# Two rocprofv3 --pmc passes (SQ stall/issue counters; MFMA / LDS / HBM-fetch
# counters) over tools/probe_kernels.py for each op named on the command line
# (default: the hot kernels).  Summarise with tools/pmc_table.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE FETCH_SIZE"
OPS=${@:-wgrad_bert attn_bwd conv_fwd_3x3_14}
for op in $OPS; do
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $R/gpurun_out/pmc_$op/p1 -o x -- python3 $R/tools/probe_kernels.py $op > $R/gpurun_out/pmc_${op}_1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $R/gpurun_out/pmc_$op/p2 -o x -- python3 $R/tools/probe_kernels.py $op > $R/gpurun_out/pmc_${op}_2.log 2>&1
done
