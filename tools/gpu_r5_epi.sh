#!/bin/bash
# Re-measure the GELU-in-epilogue fusions on the final round-5 GEMMs: BERT-base, 2 interleaved rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/epi; mkdir -p $O
for r in 1 2; do
  for v in "0 0" "1 0" "0 1" "1 1"; do
    set -- $v
    KFA_FFN_GELU_EPI=$1 KFA_DACT_EPI=$2 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/b_$1$2_$r.log 2> $O/b_$1$2_$r.err || { tail -20 $O/b_$1$2_$r.err; exit 1; }
    echo "GELU_EPI=$1 DACT_EPI=$2 r$r $(tail -1 $O/b_$1$2_$r.log | cut -c1-120)"
  done
done
