#!/bin/bash
# Overlapped per-bucket optimizer (KFA_OPT_OVERLAP): GPU test, then BERT-base A/B (3 interleaved rounds), W&D + ResNet once each
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/ovl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_opt_overlap_gpu.py -x -q --timeout 240 --timeout-method thread > $O/test.log 2>&1; rc=$?
tail -3 $O/test.log; [[ $rc -eq 0 ]] || { tail -30 $O/test.log; exit 1; }
for r in 1 2 3; do
  for v in 0 1; do
    KFA_OPT_OVERLAP=$v timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/bert_${v}_$r.log 2> $O/bert_${v}_$r.err || { tail -20 $O/bert_${v}_$r.err; exit 1; }
    echo "BERT OVL=$v r$r $(tail -1 $O/bert_${v}_$r.log | cut -c1-150)"
  done
done
for v in 0 1; do
  KFA_OPT_OVERLAP=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > $O/wd_$v.log 2> $O/wd_$v.err || { tail -20 $O/wd_$v.err; exit 1; }
  echo "WD OVL=$v $(tail -1 $O/wd_$v.log | cut -c1-150)"
  KFA_OPT_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r50_$v.log 2> $O/r50_$v.err || { tail -20 $O/r50_$v.err; exit 1; }
  echo "R50 OVL=$v $(tail -1 $O/r50_$v.log | cut -c1-150)"
done
