#!/bin/bash
# W&D world-1 fused lookup + input assembly (kfa_wd_gather_fwd): GPU tests, then the
# whole-step A/B against the lookup + assembly pair (KFA_WD_FUSED_LOOKUP=0), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdl; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_widedeep_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in 0 1; do
  KFA_WD_FUSED_LOOKUP=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/l$v$i.log 2> $O/l$v$i.err || { tail -20 $O/l$v$i.err; exit 1; }
  echo "fused_lookup=$v $(tail -1 $O/l$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("config",{}).get("loss"))')"
done
done
