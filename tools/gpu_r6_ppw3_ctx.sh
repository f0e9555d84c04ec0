#!/bin/bash
# Kernel trace of BERT-base with the FFN-down forward forced onto ppw192 (tools/routes_ab/p3072.json):
# per-dispatch durations of gemm_ppw3_kernel in the forward vs the backward of the same step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6ctx; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
KFA_ROUTES_FILE=$R/tools/routes_ab/p3072.json timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p3072 -o run -- \
  python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 6 --warmup 4 > $O/p3072.log 2> $O/p3072.err
