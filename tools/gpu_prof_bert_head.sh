#!/bin/bash
# rocprofv3 kernel trace of the BERT-base 256x128 step at HEAD, summarised to gpurun_out/profb_head.md.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profb_head -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/profb_head.log 2>&1 || { tail -20 $R/gpurun_out/profb_head.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profb_head.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/profb_head/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 1x MI355X (HEAD)" adam_kernel > gpurun_out/profb_head.md
sed -n 1,32p gpurun_out/profb_head.md
