#!/bin/bash
# BERT-base kernel traces: committed routing table vs the table with the ppw192 dgrad picks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r6bprof; mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = new ]; then export KFA_ROUTES_FILE=$R/gpurun_out/r6bert/merged.json; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o b \
    -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 > $R/$O/$v.log 2>&1 || { tail -20 $R/$O/$v.log; exit 1; }
done
cd $R
for v in old new; do
  ms=$(python3 -c "import json;print([json.loads(l) for l in open('$O/$v.log') if l.startswith('{')][-1]['ms_per_step'])")
  python3 tools/profile_summary.py $(ls $O/$v/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base $v table" adam_kernel > $O/$v.md
  rm -f $O/$v/*kernel_trace.csv
  echo "== $v"; head -36 $O/$v.md | tail -28 | cut -c1-160
done
