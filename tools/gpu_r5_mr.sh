#!/bin/bash
# multi-rank rehearsal on one GPU (2 ranks, gloo) of the driver's bench.py --gpus 2 path
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
KFA_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/mr2.log 2> gpurun_out/mr2.err || { tail -30 gpurun_out/mr2.err; exit 1; }
tail -1 gpurun_out/mr2.log | cut -c1-600
grep -i "comm\|fallback\|native" gpurun_out/mr2.err | head -5
