#!/bin/bash
# batched weight transpose (64x64 vector tiles): test, in-step time, BERT A/B of the route tables, ResNet
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6tp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "batched_weight_transpose" tests/test_gemm_ppp_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for v in r5 head; do
  f=kubeflow_controller_amd/ops/routes_gfx950.json; [ $v = r5 ] && f=kubeflow_controller_amd/ops/routes_gfx950_r5.json
  KFA_ROUTES_FILE=$R/$f timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/$v$i.log 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
  echo "$v $(tail -1 $O/$v$i.log | cut -c60-140)"
done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/r50.log 2> $O/r50.err || { tail -20 $O/r50.err; exit 1; }
echo "R50 $(tail -1 $O/r50.log | cut -c60-200)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/t -o b -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 > $R/$O/t.log 2>&1 || { tail -20 $R/$O/t.log; exit 1; }
cd $R; python3 tools/trace_calls.py $(ls $O/t/*kernel_trace.csv | head -1) 4 adam_kernel weight_transpose_multi gemm_ppw3; rm -f $O/t/*kernel_trace.csv
