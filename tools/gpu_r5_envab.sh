#!/bin/bash
# ResNet-50 env A/B, interleaved: default vs each ENVAB_SETS entry (space-separated VAR=VALUE[,VAR=VALUE])
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for i in 1 2; do
  r=$(timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>gpurun_out/envab.err | tail -1) || { tail -20 gpurun_out/envab.err; exit 1; }
  echo "default $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  for s in $ENVAB_SETS; do
    r=$(env ${s//,/ } timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>gpurun_out/envab.err | tail -1) || { tail -20 gpurun_out/envab.err; exit 1; }
    echo "$s $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
