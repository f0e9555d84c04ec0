#!/bin/bash
# A/B: BatchNorm apply-pass grid cap (KFA_BN_APPLY_BLOCKS 4096 default, 8192, 16384), ResNet-50, 3 rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/bnblocks; mkdir -p $O
for r in 1 2; do
  for v in 16384 32768 65536; do
    KFA_BN_APPLY_BLOCKS=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r_${v}_$r.log 2> $O/r_${v}_$r.err || { tail -20 $O/r_${v}_$r.err; exit 1; }
    echo "BLOCKS=$v r$r $(tail -1 $O/r_${v}_$r.log | cut -c1-110)"
  done
done
