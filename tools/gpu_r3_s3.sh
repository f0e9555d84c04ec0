#!/bin/bash
# Controller-driven ResNet-50 TFJob next to bench.py on one box, then BERT
# KFA_GEMM=auto vs fused (FFN-up bias+GELU and FFN-down dgrad GELU' epilogues).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ev_bench.log 2> gpurun_out/ev_bench.err \
  || { tail -20 gpurun_out/ev_bench.err; exit 1; }
tail -1 gpurun_out/ev_bench.log
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 60 \
  > gpurun_out/tfjob_r50.log 2> gpurun_out/tfjob_r50.err || { tail -20 gpurun_out/tfjob_r50.err; exit 1; }
tail -1 gpurun_out/tfjob_r50.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 | tail -1
bash tools/gpu_ab_bert.sh "KFA_GEMM=auto" "KFA_GEMM=fused"
