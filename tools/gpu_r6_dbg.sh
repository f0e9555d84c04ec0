#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6dbg; mkdir -p $O
KFA_ROUTES_FILE=$R/gpurun_out/r6bert/merged.json KFA_ROUTES_DUMP=$R/$O/dump.json KFA_ROUTES_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 3 --warmup 2 > $O/b.log 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
grep "kfa routes" $O/b.err | cut -c1-250
python3 -c "
import json; d=json.load(open('$O/dump.json'))
for k,v in sorted(d['routes'].items()):
  if 'proj' in k or 'dense' in k or 'ffn' in k: print(k, v)
"
