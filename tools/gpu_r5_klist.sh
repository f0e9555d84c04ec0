#!/bin/bash
# Kernel lists of the ResNet-50 and BERT-base steps on this box (run on two boxes, diff the lists)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${KLIST_TAG:-a}
mkdir -p $R/gpurun_out/klist_$tag
( hostname; rocm-smi --showserial 2>/dev/null | grep -i serial | head -2 ) > $R/gpurun_out/klist_$tag/box.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/klist_$tag/r50 -o r \
  -- python3 $R/bench.py --steps 4 --warmup 4 > $R/gpurun_out/klist_$tag/r50.log 2>&1 || { tail -20 $R/gpurun_out/klist_$tag/r50.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/klist_$tag/bert -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 4 --warmup 4 \
  > $R/gpurun_out/klist_$tag/bert.log 2>&1 || { tail -20 $R/gpurun_out/klist_$tag/bert.log; exit 1; }
cd $R
python3 tools/kernel_list.py $(ls gpurun_out/klist_$tag/r50/*kernel_trace.csv | head -1) 8 > gpurun_out/klist_$tag/r50.txt
python3 tools/kernel_list.py $(ls gpurun_out/klist_$tag/bert/*kernel_trace.csv | head -1) 8 > gpurun_out/klist_$tag/bert.txt
rm -f gpurun_out/klist_$tag/r50/*kernel_trace.csv gpurun_out/klist_$tag/bert/*kernel_trace.csv
cat gpurun_out/klist_$tag/box.txt; wc -l gpurun_out/klist_$tag/*.txt
