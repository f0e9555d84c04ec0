#!/bin/bash
# last round-5 HEAD numbers: ResNet-50 bench x2, TFJob through the controller, BERT-base, W&D
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/last; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r50_$r.log 2> $O/r50_$r.err || { tail -20 $O/r50_$r.err; exit 1; }
  echo "R50 r$r $(tail -1 $O/r50_$r.log | cut -c1-120)"
done
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 80 > $O/tfjob.log 2> $O/tfjob.err || { tail -20 $O/tfjob.err; exit 1; }
echo "TFJOB $(tail -1 $O/tfjob.log | cut -c1-200)"
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/bert.log 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
echo "BERT $(tail -1 $O/bert.log | cut -c1-120)"
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > $O/wd.log 2> $O/wd.err || { tail -20 $O/wd.err; exit 1; }
echo "WD $(tail -1 $O/wd.log | cut -c1-120)"
