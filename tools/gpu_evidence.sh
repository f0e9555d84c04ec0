#!/bin/bash
# Evidence refresh: smoke(), the controller-driven ResNet-50 TFJob (1 worker) next
# to bench.py on the same box, and a rocprofv3 trace of the BERT-base step with the
# default per-shape GEMM routing (KFA_GEMM=auto).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ev_bench.log 2> gpurun_out/ev_bench.err \
  || { tail -20 gpurun_out/ev_bench.err; exit 1; }
tail -1 gpurun_out/ev_bench.log
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 60 \
  > gpurun_out/tfjob_r50.log 2> gpurun_out/tfjob_r50.err || { tail -20 gpurun_out/tfjob_r50.err; exit 1; }
tail -1 gpurun_out/tfjob_r50.log
cd /tmp && export TMPDIR=/tmp
KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profb_auto -o b \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
  > $R/gpurun_out/profb_auto.log 2>&1 || { tail -20 $R/gpurun_out/profb_auto.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profb_auto.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/profb_auto/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 KFA_GEMM=auto (HEAD)" adam_kernel > gpurun_out/profb_auto.md
head -50 gpurun_out/profb_auto.md
