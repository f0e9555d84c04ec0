#!/bin/bash
# Same-box ResNet-50 A/B over several environment settings, interleaved:
#   gpurun -- bash tools/gpu_ab_multi.sh ROUNDS "KFA_X=0" "KFA_X=1 KFA_Y=2" ...   ("-" = no change)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/abm
N=$1; shift
for i in $(seq 1 $N); do
  k=0
  for e in "$@"; do
    k=$((k+1)); [[ "$e" == "-" ]] && e="KFA_AB_NOP=1"
    r=$(env $e timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 2>gpurun_out/abm/$k.err | tail -1) \
      || { tail -20 gpurun_out/abm/$k.err; exit 1; }
    echo "$k ($e) $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
