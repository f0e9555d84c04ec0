#!/bin/bash
# bias_act_bwd: the N-dependent default (256 rows per block for N <= 512, else 64) vs 64 everywhere; W&D + BERT
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6barpb2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "bias_act or dense or widedeep or wd_" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in default 64; do
  e=""; [ $v = 64 ] && e="KFA_BIAS_ACT_RPB=64"
  env $e timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/w$v$i.log 2> $O/w$v$i.err || { tail -20 $O/w$v$i.err; exit 1; }
  echo "wd rpb=$v $(tail -1 $O/w$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
