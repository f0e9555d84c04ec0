#!/bin/bash
# rocprofv3 PMC passes (MFMA busy, LDS bank conflicts, waits, HBM bytes) over the
# round-3 kernels (tools/pmc_r4_run.py); one counter set per pass, each pass in its
# own time limit; table -> gpurun_out/pmc_r4/table.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc_r4
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_r4/p$i -o p \
    -- python3 $R/tools/pmc_r4_run.py > $R/gpurun_out/pmc_r4/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_r4/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_table.py $(ls gpurun_out/pmc_r4/p*/*counter_collection.csv) > gpurun_out/pmc_r4/table.txt
head -120 gpurun_out/pmc_r4/table.txt
