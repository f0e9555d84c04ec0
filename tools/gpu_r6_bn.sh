#!/bin/bash
# BatchNorm pass rates per shape vs torch.add, then interleaved ResNet-50 A/B of an
# in-tree variant build (KFA_KERNELS_SO=$1, e.g. _hip_kernels_bn4.so: -DKFA_BN_ROWS=4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6bn; mkdir -p $O; V=${1:-_hip_kernels_bn4.so}
for so in _hip_kernels.so $V; do
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u tools/bench_bn_passes.py > $O/passes_$so.md 2> $O/passes_$so.err || { tail -20 $O/passes_$so.err; exit 1; }
done
for i in 1 2 3; do
for so in _hip_kernels.so $V; do
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/b_$so$i.log 2> $O/b_$so$i.err || { tail -20 $O/b_$so$i.err; exit 1; }
  echo "$so $(tail -1 $O/b_$so$i.log | cut -c1-160)"
done
done
