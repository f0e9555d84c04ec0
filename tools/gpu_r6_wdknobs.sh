#!/bin/bash
# W&D runtime defaults re-checked at HEAD: sparse-sort overlap off (KFA_SPARSE_OVERLAP=0), weight
# gradients on the side stream (KFA_SIDE_STREAM=1), per-bucket optimizer overlap (KFA_OPT_OVERLAP=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdk; mkdir -p $O
for i in 1 2; do
for v in default KFA_SPARSE_OVERLAP=0 KFA_SIDE_STREAM=1 KFA_OPT_OVERLAP=1; do
  e=""; [ $v != default ] && e=$v
  env $e timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/k.log 2> $O/k.err || { tail -20 $O/k.err; exit 1; }
  echo "$v $(tail -1 $O/k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
