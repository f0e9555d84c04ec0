#!/bin/bash
# W&D kernel trace at HEAD (rocprofv3 --kernel-trace --stats) -> profile summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wd; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/wt -o w \
  -- python3 $R/tools/bench_model.py --model wide_deep --batch 65536 --steps 10 --warmup 5 > $R/$O/wd_trace.log 2>&1 || { tail -20 $R/$O/wd_trace.log; exit 1; }
cd $R
ms=$(python3 -c "import json;print([json.loads(l) for l in open('$O/wd_trace.log') if l.startswith('{')][-1]['ms_per_step'])")
python3 tools/profile_summary.py $(ls $O/wt/*kernel_trace.csv | head -1) 10 "$ms" "Wide&Deep batch 65536 1x MI355X (round-6 HEAD)" adam_kernel > $O/wd.md
rm -f $O/wt/*kernel_trace.csv
head -40 $O/wd.md
