#!/bin/bash
# lockstep wgrad_kernel with asm transposed reads: correctness, per-shape lockstep
# microbench (KFA_WGRAD_PP=0) vs the HEAD build, ResNet-50 same-box A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/wgls; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py tests/test_gemm_gpu.py tests/test_e2e_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ab new; do
  so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
  KFA_WGRAD_PP=0 KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_wgrad_pp.py > $O/wg_$v.txt 2>&1 || { tail -20 $O/wg_$v.txt; exit 1; }
done
paste -d'|' $O/wg_ab.txt $O/wg_new.txt | grep PP= | awk -F'|' '{split($1,a," "); split($2,b," "); printf "%-20s %8s -> %8s us\n", a[2], a[3], b[3]}'
ABSO=_hip_kernels_ab.so timeout -k 10 900 bash tools/gpu_ab_so.sh
