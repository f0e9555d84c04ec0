#!/bin/bash
# conv_pp epilogue prefetch (KFA_CONV_PP_PIPE): numerics, then interleaved ResNet-50 A/B
# against an in-tree build of the same sources with -DKFA_CONV_PP_PIPE=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6pipe; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/conv_tests.log 2>&1 || { tail -30 $O/conv_tests.log; exit 1; }
tail -2 $O/conv_tests.log
for i in 1 2 3; do
for v in nopipe pipe; do
  so=_hip_kernels.so; [ $v = nopipe ] && so=_hip_kernels_nopipe.so
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/$v$i.log 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | cut -c1-200)"
done
done
