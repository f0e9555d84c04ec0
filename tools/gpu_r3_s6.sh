#!/bin/bash
# BERT-base trace on one stream (default since the side-stream A/B) + transformer tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tf_tests.log 2>&1 || { tail -30 gpurun_out/tf_tests.log; exit 1; }
tail -1 gpurun_out/tf_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profb_1s -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/profb_1s.log 2>&1 || { tail -20 $R/gpurun_out/profb_1s.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profb_1s.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/profb_1s/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128, one stream (HEAD)" adam_kernel > gpurun_out/profb_1s.md
head -45 gpurun_out/profb_1s.md
