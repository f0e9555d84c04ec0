#!/bin/bash
# Same-box A/B of the BERT-base step (256 x 128) between two environment settings, 3 rounds.
#   gpurun -- bash tools/gpu_ab_bert.sh "KFA_X=0" "KFA_X=1"
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
A="$1"; B="$2"; shift 2
for i in 1 2 3; do
  for v in A B; do
    if [[ $v == A ]]; then e="$A"; else e="$B"; fi
    r=$(env $e timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 \
      --warmup 3 "$@" 2>gpurun_out/abb_$v.err | tail -1) || { tail -20 gpurun_out/abb_$v.err; exit 1; }
    echo "$v ($e) $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
