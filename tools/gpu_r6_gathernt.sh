#!/bin/bash
# W&D lookup gather with non-temporal table loads (KFA_WD_GATHER_NT=1) vs default: tests + W&D A/B
# (the non-temporal variant and its knob were reverted after this A/B: docs/kernels.md)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6gnt; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_widedeep_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in 1 0; do
  KFA_WD_GATHER_NT=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/s$v$i.log 2> $O/s$v$i.err || { tail -20 $O/s$v$i.err; exit 1; }
  echo "gather_nt=$v $(tail -1 $O/s$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
