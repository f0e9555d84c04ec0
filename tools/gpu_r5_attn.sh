#!/bin/bash
# Attention VALU diet: attention / transformer GPU tests, the attention microbench,
# the BERT-base step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_attn_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_attn_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_attn_tests.log; exit 1; }
timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/r5_attn_bench.log 2>&1 || { tail -20 gpurun_out/r5_attn_bench.log; exit 1; }
tail -1 gpurun_out/r5_attn_bench.log
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 > gpurun_out/r5_attn_bert.log 2> gpurun_out/r5_attn_bert.err || { tail -20 gpurun_out/r5_attn_bert.err; exit 1; }
tail -1 gpurun_out/r5_attn_bert.log
