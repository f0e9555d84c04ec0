#!/bin/bash
# W&D glue removal: GPU tests of the head / input kernels, then W&D whole-step A/B
# (this tree vs the previous commit's tree built in _ab_base/), 3 interleaved rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_widedeep_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
for v in base new; do
  d=$R; [ $v = base ] && d=$R/_ab_base
  (cd $d && timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 > $R/$O/$v$i.log 2> $R/$O/$v$i.err) || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("config",{}).get("loss"))')"
done
done
