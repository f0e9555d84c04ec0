#!/bin/bash
# gemm_ppw_kernel k-loop segment shares (stamp builds 1 and 2) on the BERT-base shapes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/pwst; mkdir -p $O
for v in pw1 pw2; do
  KFA_KERNELS_SO=_hip_kernels_$v.so timeout -k 10 180 python3 -u tools/ppw_stamps.py > $O/$v.txt 2>&1 || { tail -20 $O/$v.txt; exit 1; }
  grep -v amdgpu.ids $O/$v.txt
done
