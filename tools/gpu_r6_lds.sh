#!/bin/bash
# Conflict-free LDS block reductions (BN partial / rstats passes, LN backward, bias-act
# backward): numerics, LDS bank-conflict counters of the ResNet-50 and BERT-base steps,
# interleaved A/B against the previous layout (in-tree build _hip_kernels_oldlds.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6lds; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for so in _hip_kernels_oldlds.so _hip_kernels.so; do
  KFA_KERNELS_SO=$so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $R/$O/pr_$so -o p -- python3 $R/bench.py --steps 2 --warmup 2 > $R/$O/pr_$so.log 2>&1 || { tail -5 $R/$O/pr_$so.log; exit 1; }
  KFA_KERNELS_SO=$so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $R/$O/pb_$so -o p -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 2 --warmup 2 > $R/$O/pb_$so.log 2>&1 || { tail -5 $R/$O/pb_$so.log; exit 1; }
done
cd $R
for i in 1 2; do
for so in _hip_kernels_oldlds.so _hip_kernels.so; do
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/r_$so$i.log 2> $O/r_$so$i.err || { tail -20 $O/r_$so$i.err; exit 1; }
  echo "R50 $so $(tail -1 $O/r_$so$i.log | cut -c1-130)"
  KFA_KERNELS_SO=$so timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/b_$so$i.log 2> $O/b_$so$i.err || { tail -20 $O/b_$so$i.err; exit 1; }
  echo "BERT $so $(tail -1 $O/b_$so$i.log | cut -c1-130)"
done
done
