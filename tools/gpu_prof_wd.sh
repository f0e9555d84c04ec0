#!/bin/bash
# Kernel trace of the Wide&Deep step (batch 65,536, 1 GPU) -> gpurun_out/profwd.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profwd -o wd \
  -- python3 $R/tools/bench_model.py --model wide_deep --batch 65536 --steps 10 --warmup 5 > $R/gpurun_out/profwd.log 2>&1 \
  || { tail -20 $R/gpurun_out/profwd.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profwd.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/profwd/*kernel_trace.csv | head -1) 10 "$ms" \
  "Wide&Deep batch 65536 1x MI355X (HEAD)" adam_kernel > gpurun_out/profwd.md && head -30 gpurun_out/profwd.md
