#!/bin/bash
# ResNet-50 step PMC pass at round-6 HEAD -> derived per-kernel table (MFMA busy, LDS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6r50pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/$O/p -o p \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/$O/pmc.log 2>&1 || { tail -5 $R/$O/pmc.log; exit 1; }
cd $R
python3 tools/pmc_derived.py $(ls $O/p/*counter_collection.csv) > $O/r50_pmc.md
rm -f $O/p/*counter_collection.csv
head -24 $O/r50_pmc.md
