#!/bin/bash
# wgrad split-K reduce with adaptive split-lanes: numerics, interleaved ResNet-50 A/B
# against the previous reduce (in-tree build _hip_kernels_oldred.so), per-kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6red; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for so in _hip_kernels_oldred.so _hip_kernels.so; do
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/b_$so$i.log 2> $O/b_$so$i.err || { tail -20 $O/b_$so$i.err; exit 1; }
  echo "$so $(tail -1 $O/b_$so$i.log | cut -c1-150)"
done
done
export TMPDIR=/tmp
for so in _hip_kernels_oldred.so _hip_kernels.so; do
  KFA_KERNELS_SO=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$so -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof_$so.log 2>&1 || { tail -20 $O/prof_$so.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -E "wgrad_reduce|Name" $f | cut -c1-200; done
