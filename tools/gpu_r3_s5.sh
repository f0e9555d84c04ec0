#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_widedeep_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wd_tests.log 2>&1 || { tail -30 gpurun_out/wd_tests.log; exit 1; }
tail -1 gpurun_out/wd_tests.log
for i in 1 2 3; do for v in 0 1; do
  r=$(KFA_WD_PAD64=$v timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 1
  echo "W&D pad64=$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 5 --warmup 2 2>&1 | grep "gemm tune" | head -20
timeout -k 10 300 python -u tools/bench_ppp.py 32768x2304x768 32768x3072x768 32768x768x3072 2>&1 | grep -v amdgpu.ids
