#!/bin/bash
# gemm_ppp: correctness vs fp32, then timing vs hipBLASLt / per-tile ping-pong.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gemm_ppp_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ppp_tests.log 2>&1 || { tail -30 gpurun_out/ppp_tests.log; exit 1; }
tail -2 gpurun_out/ppp_tests.log
timeout -k 10 240 python -u tools/bench_ppp.py "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_ppp.log
