#!/bin/bash
# ResNet-50 whole-step A/B: committed table vs every conv decision within 4 % flipped to its runner-up
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6r50ab; mkdir -p $O
for i in 1 2 3; do
for v in base r50_flip_close; do
  f=$R/kubeflow_controller_amd/ops/routes_gfx950.json; [ $v != base ] && f=$R/tools/routes_ab/$v.json
  KFA_ROUTES_FILE=$f timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/$v$i.log 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["routes"]["timed"])')"
done
done
