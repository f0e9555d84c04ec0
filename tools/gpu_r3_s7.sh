#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k wgrad \
  > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
bash tools/gpu_ab_bert_so.sh
for i in 1 2; do for v in 0 1; do
  r=$(KFA_WGRAD_PP=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 1
  echo "W&D wgrad_pp=$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
