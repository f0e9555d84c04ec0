#!/bin/bash
# A/B: conv persistent-grid cap (KFA_CONV_OVERSUB 0 = one block per tile, 1 = 2 blocks/CU default, 2 = 4 blocks/CU), ResNet-50, 2 rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/oversub; mkdir -p $O
for r in 1 2; do
  for v in 1 0 2; do
    KFA_CONV_OVERSUB=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r_${v}_$r.log 2> $O/r_${v}_$r.err || { tail -20 $O/r_${v}_$r.err; exit 1; }
    echo "OVERSUB=$v r$r $(tail -1 $O/r_${v}_$r.log | cut -c1-110)"
  done
done
