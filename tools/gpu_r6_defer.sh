#!/bin/bash
# Deferred split-K weight-gradient reduces: tests, then interleaved ResNet-50 and BERT-base
# A/B (KFA_DEFER_WGRAD_REDUCE=0 vs default on), then a ResNet kernel trace of the new form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6defer; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py -k "deferred or wgrad" tests/test_transformer_gpu.py tests/test_opt_overlap_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
for v in 0 1; do
  KFA_DEFER_WGRAD_REDUCE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/r$v$i.log 2> $O/r$v$i.err || { tail -20 $O/r$v$i.err; exit 1; }
  echo "R50 defer=$v $(tail -1 $O/r$v$i.log | cut -c85-125)"
done
done
for i in 1 2; do
for v in 0 1; do
  KFA_DEFER_WGRAD_REDUCE=$v timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/b$v$i.log 2> $O/b$v$i.err || { tail -20 $O/b$v$i.err; exit 1; }
  echo "BERT defer=$v $(tail -1 $O/b$v$i.log | cut -c70-115)"
done
done
