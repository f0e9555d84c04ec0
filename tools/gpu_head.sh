#!/bin/bash
# HEAD evidence (gpurun --timeout 1100 -- bash tools/gpu_head.sh): GPU tests, ResNet-50 bench + rocprof trace, BERT-base bench + trace, W&D bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>/dev/null | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 2>/dev/null | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o r50 \
  -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof.log 2>&1 || { tail -20 $R/gpurun_out/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profb_fin -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/profb_fin.log 2>&1 || { tail -20 $R/gpurun_out/profb_fin.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/prof.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/prof/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 bs256 1x MI355X (round-3 HEAD)" > gpurun_out/prof_summary.md
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profb_fin.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/profb_fin/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 1x MI355X (round-3 HEAD)" adam_kernel > gpurun_out/profb_fin.md
head -12 gpurun_out/prof_summary.md; head -12 gpurun_out/profb_fin.md
