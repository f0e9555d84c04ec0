#!/bin/bash
# BERT-base (256 x 128) with the dense projections on hipBLASLt vs on the
# hand-written GEMMs (KFA_GEMM=1: all projections; fused: only the epilogue-fused
# FFN-up forward / dgrad and the activation denses), interleaved.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for cfg in "KFA_GEMM=0" "KFA_GEMM=1" "KFA_GEMM=fused" "KFA_GEMM=0" "KFA_GEMM=1" "KFA_GEMM=fused"; do
  r=$(env $cfg timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 \
    2> gpurun_out/bert_gemm.err | tail -1) || { tail -20 gpurun_out/bert_gemm.err; exit 1; }
  echo "$cfg $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
