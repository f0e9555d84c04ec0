#!/bin/bash
# Sparse-update kernels on 1 GPU: numerics tests, the W&D-shaped micro-bench
# (segment-reduce vs atomic), then Wide&Deep b65536 end to end in both modes.
#   gpurun -- bash tools/gpu_sparse.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sparse_gpu.py tests/test_transformer_gpu.py \
  tests/test_widedeep_gpu.py > gpurun_out/sparse_tests.log 2>&1 || { tail -40 gpurun_out/sparse_tests.log; exit 1; }
tail -2 gpurun_out/sparse_tests.log
timeout -k 10 300 python -u tools/bench_sparse.py > gpurun_out/bench_sparse.log 2>&1 \
  || { tail -30 gpurun_out/bench_sparse.log; exit 1; }
cat gpurun_out/bench_sparse.log
for mode in 0 1 0 1; do
  KFA_SPARSE_ATOMIC=$mode timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 \
    --warmup 5 > gpurun_out/wd_$mode.log 2> gpurun_out/wd_$mode.err || { tail -30 gpurun_out/wd_$mode.err; exit 1; }
  echo "W&D atomic=$mode $(tail -1 gpurun_out/wd_$mode.log)"
done
[[ ${PROF:-0} == 1 ]] && bash tools/gpu_prof_wd.sh > gpurun_out/pw.txt 2>&1
exit 0
