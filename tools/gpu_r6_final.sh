#!/bin/bash
# Round-6 HEAD evidence: the driver's check (GPU tests, smoke, bench), BERT-base /
# W&D benches, BERT + ResNet kernel traces, a BERT PMC pass, the TFJob-through-controller ResNet
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; O=gpurun_out/r6final; mkdir -p $O
bash tools/gpu_r6_check.sh || exit 1
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/bert.log 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
tail -1 $O/bert.log | cut -c1-220
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > $O/wd.log 2> $O/wd.err || { tail -20 $O/wd.err; exit 1; }
tail -1 $O/wd.log | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/bt -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 > $R/$O/bert_trace.log 2>&1 || { tail -20 $R/$O/bert_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rt -o r \
  -- python3 $R/bench.py --steps 10 --warmup 5 > $R/$O/r50_trace.log 2>&1 || { tail -20 $R/$O/r50_trace.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/$O/bp -o p \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 2 --warmup 2 > $R/$O/bert_pmc.log 2>&1 || { tail -5 $R/$O/bert_pmc.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('$O/bert_trace.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls $O/bt/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 1x MI355X (round-6 HEAD)" adam_kernel > $O/bert.md
ms=$(python3 -c "import json;print([json.loads(l) for l in open('$O/r50_trace.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls $O/rt/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 bs256 1x MI355X (round-6 HEAD)" > $O/r50.md
python3 tools/pmc_derived.py $(ls $O/bp/*counter_collection.csv) > $O/bert_pmc.md || true
python3 tools/kernel_list.py $(ls $O/rt/*kernel_trace.csv | head -1) 15 > $O/r50_klist.txt
python3 tools/kernel_list.py $(ls $O/bt/*kernel_trace.csv | head -1) 8 > $O/bert_klist.txt
rm -f $O/bt/*kernel_trace.csv $O/rt/*kernel_trace.csv $O/bp/*counter_collection.csv
head -30 $O/bert.md | tail -22
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 80 > $O/tfjob_r50.log 2> $O/tfjob_r50.err || { tail -20 $O/tfjob_r50.err; exit 1; }
tail -1 $O/tfjob_r50.log | cut -c1-300
