#!/bin/bash
# PMC counters of pp (main loop probe) vs gemm_ppp (no-store probe), one pass per counter set.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc_ppp
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_ppp/p$i -o p \
    -- python3 $R/tools/pmc_ppp_run.py > $R/gpurun_out/pmc_ppp/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_ppp/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_table.py $(ls gpurun_out/pmc_ppp/p*/*counter_collection.csv) | tee gpurun_out/pmc_ppp/table.txt
