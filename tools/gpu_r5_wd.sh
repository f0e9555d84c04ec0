#!/bin/bash
# W&D HEAD kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r5wd
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5wd/t -o w \
  -- python3 $R/tools/bench_model.py --model wide_deep --batch 65536 --steps 10 --warmup 5 \
  > $R/gpurun_out/r5wd/wd.log 2>&1 || { tail -20 $R/gpurun_out/r5wd/wd.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/r5wd/wd.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls gpurun_out/r5wd/t/*kernel_trace.csv | head -1) 10 "$ms" "Wide&Deep batch 65536 1x MI355X (round-5 HEAD)" adam_kernel > gpurun_out/r5wd/wd.md
head -45 gpurun_out/r5wd/wd.md
