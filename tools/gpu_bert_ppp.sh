#!/bin/bash
# BERT-base 256x128 with the projections on per-shape auto routing (KFA_GEMM=auto:
# persistent MFMA GEMM where it measured faster than hipBLASLt) vs all-library
# (KFA_GEMM=0), interleaved on one box; the tuner's choices are logged.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_ppp_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/bert_ppp_tests.log 2>&1 || { tail -30 gpurun_out/bert_ppp_tests.log; exit 1; }
tail -1 gpurun_out/bert_ppp_tests.log
for i in 1 2; do for g in auto 0; do
  KFA_GEMM=$g KFA_GEMM_TUNE_LOG=1 timeout -k 10 240 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 \
    --steps 20 --warmup 5 > gpurun_out/bert_$g.log 2> gpurun_out/bert_$g.err || { tail -20 gpurun_out/bert_$g.err; exit 1; }
  echo "KFA_GEMM=$g $(python3 -c "import json;d=json.loads(open('gpurun_out/bert_$g.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done; done
grep "gemm tune" gpurun_out/bert_auto.err | sort -u | cut -c1-160
