#!/bin/bash
# (1) CU-hog throughput probe per KFA_CONV_OVERSUB mode; (2) HEAD kernel traces of the
# ResNet-50 and BERT-base steps; (3) PMC pass over the ResNet step (MFMA busy per kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r5prof
for m in 1 2 0; do
KFA_CONV_OVERSUB=$m timeout -k 10 240 python -u tools/probe_cu_hog_step.py --hog 0,16,32,64 > gpurun_out/r5_hog$m.log 2> gpurun_out/r5_hog$m.err || { tail -20 gpurun_out/r5_hog$m.err; exit 1; }
tail -1 gpurun_out/r5_hog$m.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5prof/r50 -o r50 \
  -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/r5prof/r50.log 2>&1 || { tail -20 $R/gpurun_out/r5prof/r50.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5prof/bert -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/r5prof/bert.log 2>&1 || { tail -20 $R/gpurun_out/r5prof/bert.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/r5prof/pmc1 -o p \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r5prof/pmc1.log 2>&1 || { tail -5 $R/gpurun_out/r5prof/pmc1.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/r5prof/r50.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/r5prof/r50/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 bs256 1x MI355X (round-5 HEAD)" > gpurun_out/r5prof/r50.md
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/r5prof/bert.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/r5prof/bert/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 1x MI355X (round-5 HEAD)" adam_kernel > gpurun_out/r5prof/bert.md
python3 tools/pmc_derived.py $(ls gpurun_out/r5prof/pmc1/*counter_collection.csv) > gpurun_out/r5prof/pmc_derived.md || true
head -16 gpurun_out/r5prof/r50.md; head -24 gpurun_out/r5prof/bert.md; head -20 gpurun_out/r5prof/pmc_derived.md
