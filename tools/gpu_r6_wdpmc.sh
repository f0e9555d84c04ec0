#!/bin/bash
# W&D step PMC pass at HEAD (MFMA busy, LDS, waves) -> derived per-kernel table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdpmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/$O/p -o p \
  -- python3 $R/tools/bench_model.py --model wide_deep --batch 65536 --steps 2 --warmup 2 > $R/$O/pmc.log 2>&1 || { tail -5 $R/$O/pmc.log; exit 1; }
cd $R
python3 tools/pmc_derived.py $(ls $O/p/*counter_collection.csv) > $O/wd_pmc.md
rm -f $O/p/*counter_collection.csv
head -20 $O/wd_pmc.md
