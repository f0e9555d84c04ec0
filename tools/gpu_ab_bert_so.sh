#!/bin/bash
# Same-box A/B of the BERT-base step: ops/_hip_kernels_ab.so (A) vs ops/_hip_kernels.so (B), 3 rounds.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [[ $v == A ]]; then so=_hip_kernels_ab.so; else so=_hip_kernels.so; fi
    r=$(KFA_KERNELS_SO=$so timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 \
      --steps 10 --warmup 3 2>gpurun_out/abb_$v.err | tail -1) || { tail -20 gpurun_out/abb_$v.err; exit 1; }
    echo "$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
