#!/bin/bash
# Mid-round HEAD check: every GPU test, smoke(), the 1-GPU ResNet bench, BERT / W&D benches
# and the BERT kernel trace after the attention diet
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out/r5head2
bash tools/gpu_r5_check.sh || exit 1
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > gpurun_out/r5head2/wd.log 2> gpurun_out/r5head2/wd.err || { tail -20 gpurun_out/r5head2/wd.err; exit 1; }
tail -1 gpurun_out/r5head2/wd.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5head2/bert -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/r5head2/bert.log 2>&1 || { tail -20 $R/gpurun_out/r5head2/bert.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/r5head2/bert.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/r5head2/bert/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 1x MI355X (round-5 HEAD, after the attention diet)" adam_kernel > gpurun_out/r5head2/bert.md
head -30 gpurun_out/r5head2/bert.md
