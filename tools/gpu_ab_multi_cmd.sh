#!/bin/bash
# Same-box A/B of any bench command over several environment settings, interleaved:
#   gpurun -- bash tools/gpu_ab_multi_cmd.sh ROUNDS "python -u tools/bench_model.py ..." "KFA_X=0" "-" ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/abmc
N=$1; CMD=$2; shift 2
for i in $(seq 1 $N); do
  k=0
  for e in "$@"; do
    k=$((k+1)); [[ "$e" == "-" ]] && e="KFA_AB_NOP=1"
    r=$(env $e timeout -k 10 300 $CMD 2>gpurun_out/abmc/$k.err | tail -1) || { tail -20 gpurun_out/abmc/$k.err; exit 1; }
    echo "$k ($e) $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
