#!/bin/bash
# BERT-base step with the attention backward re-hashing (default) vs reading the forward's mask
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_attn_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r5_attn_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_attn_tests.log; exit 1; }
for i in 1 2; do
for m in 0 1; do
  KFA_ATTN_MASK=$m timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 > gpurun_out/r5_attn_bert_m$m.log 2> gpurun_out/r5_attn_bert_m$m.err || { tail -20 gpurun_out/r5_attn_bert_m$m.err; exit 1; }
  echo "KFA_ATTN_MASK=$m $(tail -1 gpurun_out/r5_attn_bert_m$m.log | cut -c1-200)"
done
done
