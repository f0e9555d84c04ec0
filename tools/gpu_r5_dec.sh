#!/bin/bash
# tied MLM decoder backward: dlogits * g + decoder-bias column sums in one pass (KFA_DEC_SCALE_COLSUM=1) vs torch mul_ + colsum
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/dec; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_transformer_gpu.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in 0 1; do
    r=$(KFA_DEC_SCALE_COLSUM=$v timeout -k 10 300 python3 -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 2>$O/bert_$v.err | tail -1) || { tail -20 $O/bert_$v.err; exit 1; }
    echo "bert dec=$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['loss'])")"
  done
done
