#!/bin/bash
# conv_igemm gather: tap offset as one scalar add (row offset at tap (0,0)) — conv tests, then
# ResNet-50 A/B against the previous build (ops/_hip_kernels_ab.so)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_e2e_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_ig_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r5_ig_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_ig_tests.log; exit 1; }
bash tools/gpu_ab_so.sh
