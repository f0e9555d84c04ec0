#!/bin/bash
# bias_act_bwd rows per block (KFA_BIAS_ACT_RPB 64 = default / 128 / 256): W&D and BERT-base, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6barpb; mkdir -p $O
for i in 1 2; do
for v in 64 128 256; do
  KFA_BIAS_ACT_RPB=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/w$v$i.log 2> $O/w$v$i.err || { tail -20 $O/w$v$i.err; exit 1; }
  echo "wd rpb=$v $(tail -1 $O/w$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
for i in 1 2; do
for v in 64 128 256; do
  KFA_BIAS_ACT_RPB=$v timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/b$v$i.log 2> $O/b$v$i.err || { tail -20 $O/b$v$i.err; exit 1; }
  echo "bert rpb=$v $(tail -1 $O/b$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
