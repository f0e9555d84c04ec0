#!/bin/bash
# wgrad_pp_kernel k-loop segment shares from the two stamp builds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/stamps
for v in st1 st2; do
  KFA_KERNELS_SO=_hip_kernels_$v.so timeout -k 10 180 python3 -u tools/wgrad_stamps.py 32768x2304x768 32768x768x3072 32768x3072x768 32768x768x768 \
    > gpurun_out/stamps/$v.txt 2>&1 || { tail -20 gpurun_out/stamps/$v.txt; exit 1; }
  cat gpurun_out/stamps/$v.txt
done
