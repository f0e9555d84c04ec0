#!/bin/bash
# pointwise weight-gradient route after the asm-read changes: lockstep (0) / shipped rule (1) / ping-pong for every >=128-channel weight (2)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/wgrule; mkdir -p $O
for v in 0 1 2; do
  KFA_WGRAD_PP=$v timeout -k 10 300 python3 -u tools/bench_wgrad_pp.py > $O/pp$v.txt 2>&1 || { tail -20 $O/pp$v.txt; exit 1; }
done
paste -d'|' $O/pp0.txt $O/pp1.txt $O/pp2.txt | grep PP= | awk -F'|' '{split($1,a," "); split($2,b," "); split($3,c," "); printf "%-20s %8s %8s %8s us\n", a[2], a[3], b[3], c[3]}'
