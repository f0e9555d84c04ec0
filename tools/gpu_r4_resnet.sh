#!/bin/bash
# Round-4 ResNet-50 evidence: kernel trace of the bench step + per-kernel PMC passes
# (MFMA busy / instructions, LDS, HBM bytes) -> gpurun_out/prof_r4.md, gpurun_out/pmc_r50/derived.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc_r50
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o r50 \
  -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof.log 2>&1 || { tail -20 $R/gpurun_out/prof.log; exit 1; }
i=0
for set in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_r50/p$i -o p \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/pmc_r50/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_r50/p$i.log; exit 1; }
done
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/prof.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/prof/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 bs256 1x MI355X (round-4 HEAD)" > gpurun_out/prof_r4.md
python3 tools/pmc_derived.py $(ls gpurun_out/pmc_r50/p*/*counter_collection.csv) > gpurun_out/pmc_r50/derived.md
head -14 gpurun_out/prof_r4.md; head -30 gpurun_out/pmc_r50/derived.md
