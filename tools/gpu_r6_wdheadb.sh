#!/bin/bash
# W&D head backward grid: 256 blocks (default) vs 512 / 1024 (KFA_WD_HEAD_BWD_BLOCKS=256), tests + interleaved A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_widedeep_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in 256 1024 512; do
  KFA_WD_HEAD_BWD_BLOCKS=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $O/h$v$i.log 2> $O/h$v$i.err || { tail -20 $O/h$v$i.err; exit 1; }
  echo "head_bwd_blocks=$v $(tail -1 $O/h$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
