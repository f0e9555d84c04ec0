#!/bin/bash
# round-6 baseline on a fresh box: ResNet-50 bench eager vs HIP graph, BERT-base
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6base; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r50.log 2> $O/r50.err || { tail -20 $O/r50.err; exit 1; }
echo "R50 eager $(tail -1 $O/r50.log | cut -c1-160)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph auto > $O/r50g.log 2> $O/r50g.err || { tail -20 $O/r50g.err; exit 1; }
echo "R50 graph $(tail -1 $O/r50g.log | cut -c1-400)"
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/bert.log 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
echo "BERT $(tail -1 $O/bert.log | cut -c1-160)"
