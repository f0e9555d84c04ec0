#!/bin/bash
# attention backward: QKV-bias gradient from per-(sequence, wave) partial rows (KFA_ATTN_DBIAS=1) vs the column-sum pass
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/dbias; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attention_gpu.py tests/test_transformer_gpu.py tests/test_e2e_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/bench_attn.py > $O/attn.txt 2>&1 || { tail -20 $O/attn.txt; exit 1; }
grep -v amdgpu.ids $O/attn.txt | tail -12
for i in 1 2 3; do
  for v in 0 1; do
    r=$(KFA_ATTN_DBIAS=$v timeout -k 10 300 python3 -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 2>$O/bert_$v.err | tail -1) || { tail -20 $O/bert_$v.err; exit 1; }
    echo "bert dbias=$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['loss'])")"
  done
done
