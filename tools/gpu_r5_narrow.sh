#!/bin/bash
# A/B: 256x64 conv tile (variant 3) for the long-reduction 64-channel convs (KFA_CONV_NARROW_LONGK=3) vs 128x64
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/narrow; mkdir -p $O
for r in 1 2 3; do
  for v in 1 3; do
    KFA_CONV_NARROW_LONGK=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b_${v}_$r.log 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    echo "LONGK=$v r$r $(tail -1 $O/b_${v}_$r.log | cut -c1-90)"
  done
done
