#!/bin/bash
# A/B: ping-pong weight gradient on every pointwise weight >= 128x128 (KFA_WGRAD_PP=2) vs the size rule (1)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/pp2; mkdir -p $O
for r in 1 2; do
  for v in 1 2; do
    KFA_WGRAD_PP=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r_${v}_$r.log 2> $O/r_${v}_$r.err || { tail -20 $O/r_${v}_$r.err; exit 1; }
    echo "R50 PP=$v r$r $(tail -1 $O/r_${v}_$r.log | cut -c1-110)"
    KFA_WGRAD_PP=$v timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/b_${v}_$r.log 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    echo "BERT PP=$v r$r $(tail -1 $O/b_${v}_$r.log | cut -c1-110)"
  done
done
