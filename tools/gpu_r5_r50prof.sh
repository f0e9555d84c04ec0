#!/bin/bash
# ResNet-50 HEAD kernel trace + MFMA PMC pass (after the conv_igemm gather change)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r5r50
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5r50/t -o r50 \
  -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/r5r50/r50.log 2>&1 || { tail -20 $R/gpurun_out/r5r50/r50.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/r5r50/pmc -o p \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r5r50/pmc.log 2>&1 || { tail -5 $R/gpurun_out/r5r50/pmc.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/r5r50/r50.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/r5r50/t/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 bs256 1x MI355X (round-5 late HEAD, after the asm operand reads)" > gpurun_out/r5r50/r50.md
python3 tools/pmc_derived.py $(ls gpurun_out/r5r50/pmc/*counter_collection.csv) > gpurun_out/r5r50/pmc.md || true
rm -f gpurun_out/r5r50/t/*kernel_trace.csv gpurun_out/r5r50/pmc/*counter_collection.csv
head -24 gpurun_out/r5r50/r50.md; head -14 gpurun_out/r5r50/pmc.md
