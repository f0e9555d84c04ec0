#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/pwst3; mkdir -p $O
KFA_KERNELS_SO=_hip_kernels_pw3.so timeout -k 10 180 python3 -u tools/ppw_stamps.py 32768x2304x768 32768x768x3072 > $O/st.txt 2>&1 || { tail -20 $O/st.txt; exit 1; }
grep -v amdgpu.ids $O/st.txt
