#!/bin/bash
# Non-headline BASELINE configs on 1 GPU: BERT-base 256x128 and Wide&Deep b65536
# (same JSON contract as bench.py).  Each run has its own time limit; the chain
# stops at the first failure.
#   gpurun -- bash tools/gpu_models.sh [bert|wd|all]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
what=${1:-all}
if [[ $what == bert || $what == all ]]; then
  timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 \
    > gpurun_out/bert.log 2> gpurun_out/bert.err || { tail -30 gpurun_out/bert.err; exit 1; }
  echo "BERT $(tail -1 gpurun_out/bert.log)"
fi
if [[ $what == wd || $what == all ]]; then
  timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 \
    > gpurun_out/wd.log 2> gpurun_out/wd.err || { tail -30 gpurun_out/wd.err; exit 1; }
  echo "W&D $(tail -1 gpurun_out/wd.log)"
fi
