#!/bin/bash
# wgrad_pp_kernel with asm transposed reads (no compiler vmcnt(0) per phase):
# correctness, per-shape microbench vs the HEAD build (_hip_kernels_ab.so), stamps,
# then BERT-base and ResNet-50 same-box A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/wgasm; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py tests/test_gemm_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in ab new; do
  so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
  KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_wgrad_pp.py > $O/wg_$v.txt 2>&1 || { tail -20 $O/wg_$v.txt; exit 1; }
done
paste $O/wg_ab.txt $O/wg_new.txt | awk '{print $2, $3, $6, "->", $10, $13}'
KFA_KERNELS_SO=_hip_kernels_st1.so timeout -k 10 180 python3 -u tools/wgrad_stamps.py 32768x2304x768 32768x768x768 > $O/st1.txt 2>&1 || { tail -20 $O/st1.txt; exit 1; }
cat $O/st1.txt
for i in 1 2 3; do
  for v in ab new; do
    so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
    r=$(KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 2>$O/bert_$v.err | tail -1) || { tail -20 $O/bert_$v.err; exit 1; }
    echo "bert $v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
[[ -n "$WG_R50" ]] && ABSO=_hip_kernels_ab.so timeout -k 10 900 bash tools/gpu_ab_so.sh
