#!/bin/bash
# HBM bytes per kernel of the ResNet-50 step (FETCH_SIZE / WRITE_SIZE passes) + MFMA busy:
# which memory-bound kernels run below the HBM roofline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r5bytes
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/r5bytes/p$i -o p \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r5bytes/p$i.log 2>&1 || { tail -5 $R/gpurun_out/r5bytes/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_derived.py $(ls gpurun_out/r5bytes/p*/*counter_collection.csv) > gpurun_out/r5bytes/derived.md
head -60 gpurun_out/r5bytes/derived.md
