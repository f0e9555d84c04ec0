#!/bin/bash
# HEAD check: GPU test suite, ResNet-50 bench, the same model as a TFJob, Wide&Deep and BERT-base 1-GPU numbers.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>/dev/null | tail -1
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 80 \
  > gpurun_out/tfjob_r50.log 2> gpurun_out/tfjob_r50.err || { tail -20 gpurun_out/tfjob_r50.err; exit 1; }
tail -1 gpurun_out/tfjob_r50.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>/dev/null | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 2>/dev/null | tail -1
KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 5 --warmup 2 2>&1 | grep "gemm tune" | head -20
