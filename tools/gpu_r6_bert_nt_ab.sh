#!/bin/bash
# BERT-base whole-step A/B of single routing decisions (non-temporal own variants on the BERT forwards) (tables in tools/routes_ab/), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6nab; mkdir -p $O
for i in 1 2; do
for v in base n3072 n768; do
  f=$R/kubeflow_controller_amd/ops/routes_gfx950.json; [ $v != base ] && f=$R/tools/routes_ab/$v.json
  KFA_ROUTES_FILE=$f timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/$v$i.log 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["routes"])')"
done
done
