#!/bin/bash
# Same-box A/B of the ResNet-50 step between two environment settings
# (interleaved, 3 rounds):  gpurun -- bash tools/gpu_ab_env.sh "KFA_X=0" "KFA_X=1" [bench args]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
A="$1"; B="$2"; shift 2
for i in 1 2 3; do
  for v in A B; do
    if [[ $v == A ]]; then e="$A"; else e="$B"; fi
    r=$(env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" 2>gpurun_out/ab_$v.err | tail -1) \
      || { tail -20 gpurun_out/ab_$v.err; exit 1; }
    echo "$v ($e) $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
