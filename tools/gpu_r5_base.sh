#!/bin/bash
# Round-5 baseline: 1-GPU ResNet bench + per-layer conv timings (own vs MIOpen)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
rocm-smi --showclocks > gpurun_out/r5_clocks.log 2>&1 || true
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench.log 2> gpurun_out/r5_bench.err || { tail -20 gpurun_out/r5_bench.err; exit 1; }
tail -1 gpurun_out/r5_bench.log
timeout -k 10 400 python -u tools/bench_conv.py > gpurun_out/r5_conv.log 2>&1 || { tail -20 gpurun_out/r5_conv.log; exit 1; }
cat gpurun_out/r5_conv.log
