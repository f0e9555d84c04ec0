#!/bin/bash
# 512x128 ping-pong conv: numerics, per-layer A/B (igemm / pp / pp512), then the NHALF=2 epilogue A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_dgrad or stats_fused" > gpurun_out/r5_pp512_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_pp512_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_pp512_tests.log; exit 1; }
timeout -k 10 400 python -u tools/bench_conv_pp.py > gpurun_out/r5_pp512_bench.log 2>&1 || { tail -20 gpurun_out/r5_pp512_bench.log; exit 1; }
cat gpurun_out/r5_pp512_bench.log
ABSO=_hip_kernels_nh2.so bash tools/gpu_ab_so.sh
