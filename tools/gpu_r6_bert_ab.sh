#!/bin/bash
# BERT-base A/B: committed routing table vs the round-5 copy (routes_gfx950_r5.json, recreate it first:
#   git show ed33e07:kubeflow_controller_amd/ops/routes_gfx950.json > kubeflow_controller_amd/ops/routes_gfx950_r5.json), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6bab; mkdir -p $O
for i in 1 2 3; do
for v in r5 head; do
  f=kubeflow_controller_amd/ops/routes_gfx950.json; [ $v = r5 ] && f=kubeflow_controller_amd/ops/routes_gfx950_r5.json
  KFA_ROUTES_FILE=$R/$f timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/$v$i.log 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | cut -c1-300)"
done
done
