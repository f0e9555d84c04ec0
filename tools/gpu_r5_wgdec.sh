#!/bin/bash
# the BERT MLM-decoder weight gradient (5120 x 30528 x 768) on the ping-pong kernel: tests, shape timing, BERT A/B vs HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/wgdec; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ab new; do
  so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
  KFA_KERNELS_SO=$so timeout -k 10 120 python3 tools/bench_wgrad_decoder.py 2>&1 | grep PP= | sed "s/^/$v /"
done
for i in 1 2 3; do
  for v in ab new; do
    so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
    r=$(KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 2>$O/bert_$v.err | tail -1) || { tail -20 $O/bert_$v.err; exit 1; }
    echo "bert $v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
