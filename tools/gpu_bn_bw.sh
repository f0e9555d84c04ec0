#!/bin/bash
# HBM bytes per kernel of the ResNet-50 training step: two rocprofv3 --pmc passes
# (FETCH_SIZE, then WRITE_SIZE: together they exceed the 4 TCC counters of one
# pass) over a short bench.py run; tools/bw_table.py turns them into TB/s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/bw/fetch -o x \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/bw_fetch.log 2>&1 || { tail -20 $R/gpurun_out/bw_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/bw/write -o x \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/bw_write.log 2>&1 || { tail -20 $R/gpurun_out/bw_write.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d $R/gpurun_out/bw/mfma -o x -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/bw_mfma.log 2>&1 \
  || { tail -20 $R/gpurun_out/bw_mfma.log; exit 1; }
cd $R
python3 tools/pmc_summary.py gpurun_out/bw/mfma/*counter_collection.csv "ResNet-50 bs256 step: MFMA counters" \
  > gpurun_out/mfma_table.md
python3 tools/bw_table.py gpurun_out/bw/fetch/*counter_collection.csv gpurun_out/bw/write/*counter_collection.csv \
  > gpurun_out/bw_table.md && head -50 gpurun_out/bw_table.md
