#!/bin/bash
# Attention backward mask A/B: LDS-parked vs per-step memory reads; the rocprof view of both
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_attn_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r5_attn_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_attn_tests.log; exit 1; }
KFA_ATTN_MASK_LDS=0 timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_attn_tests3.log 2>&1; rc=$?
tail -1 gpurun_out/r5_attn_tests3.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_attn_tests3.log; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | tail -1 || exit 1
  KFA_ATTN_MASK_LDS=0 timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | tail -1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/attn/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $GRAFT_REPO_ROOT/gpurun_out/attn/kt.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/attn/kt.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/attn/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cat {} | cut -c1-200 | head -12
