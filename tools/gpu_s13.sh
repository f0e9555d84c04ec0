#!/bin/bash
# KFA_GEMM=auto (per-shape own-vs-library for Linear layers): GPU tests, the
# tuner's choices, and same-box A/Bs on ResNet-50 and Wide&Deep.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 2>&1 | grep -E "gemm tune|metric" | cut -c1-200
KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 5 --warmup 2 2>&1 \
  | grep -E "gemm tune|metric" | cut -c1-200
bash tools/gpu_ab_env.sh KFA_GEMM=0 KFA_GEMM=auto || exit 1
for i in 1 2; do for g in 0 auto; do
  r=$(KFA_GEMM=$g timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1)
  echo "W&D KFA_GEMM=$g $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
