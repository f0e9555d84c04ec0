#!/bin/bash
# Round-3 GEMM session: persistent GEMM tests (256- and 192-wide tiles), the
# transformer tests (two-input LN backward, own-route BERT vs fp32), then the
# per-shape timing table vs hipBLASLt.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gemm_ppp_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/gemm_r3_tests.log 2>&1 || { tail -40 gpurun_out/gemm_r3_tests.log; exit 1; }
tail -2 gpurun_out/gemm_r3_tests.log
timeout -k 10 240 python -u tools/bench_ppp.py "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/bench_ppp.log
