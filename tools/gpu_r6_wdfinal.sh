#!/bin/bash
# W&D at HEAD: fused lookup on/off A/B (3 more interleaved rounds) + the HEAD kernel trace summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdf; mkdir -p $O
for i in 1 2 3; do
for v in 1 0; do
  KFA_WD_FUSED_LOOKUP=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/l$v$i.log 2> $O/l$v$i.err || { tail -20 $O/l$v$i.err; exit 1; }
  echo "fused_lookup=$v $(tail -1 $O/l$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
bash tools/gpu_r6_wdprof.sh > $O/prof.out 2>&1 || { tail -20 $O/prof.out; exit 1; }
head -30 gpurun_out/r6wd/wd.md
