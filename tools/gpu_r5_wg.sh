#!/bin/bash
# gathered ping-pong wgrad: numerics, per-layer A/B (tools/bench_conv.py wgrad column) and ResNet bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/r5_wg_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_wg_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_wg_tests.log; exit 1; }
for v in 1 0; do
KFA_WGRAD_PP_GATHER=$v timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/r5_wg_conv$v.log 2>&1 || { tail -20 gpurun_out/r5_wg_conv$v.log; exit 1; }
grep -E "k3|s2|TOTAL" gpurun_out/r5_wg_conv$v.log | sed -E 's/\| fwd.*wgrad/| wgrad/'
done
for i in 1 2; do for v in 1 0; do
KFA_WGRAD_PP_GATHER=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_wg_b$v$i.log 2> gpurun_out/r5_wg_b$v$i.err || { tail -20 gpurun_out/r5_wg_b$v$i.err; exit 1; }
echo "GATHER=$v $(python3 -c "import json;d=json.loads(open('gpurun_out/r5_wg_b$v$i.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done; done
