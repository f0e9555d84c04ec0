#!/bin/bash
# N <= 64 tile variants per ResNet-50 layer: 128x64 (1, default) vs 256x64 (3)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
VARS=-1,3 timeout -k 10 400 python -u tools/bench_conv_pp.py > gpurun_out/r5_narrow.log 2>&1 || { tail -20 gpurun_out/r5_narrow.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_narrow.log | head -5
