#!/bin/bash
# conv ping-pong kernel: numerics tests, then per-layer A/B vs the 128x128 kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd_dgrad or stats_fused" > gpurun_out/r5_pp_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5_pp_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_pp_tests.log; exit 1; }
timeout -k 10 120 python -u -m pytest tests/test_comm_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/r5_comm_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5_comm_gpu.log; [[ $rc -eq 124 || $rc -eq 137 || $rc -ge 128 ]] && exit 1
timeout -k 10 400 python -u tools/bench_conv_pp.py > gpurun_out/r5_pp_bench.log 2>&1 || { tail -20 gpurun_out/r5_pp_bench.log; exit 1; }
cat gpurun_out/r5_pp_bench.log
