#!/bin/bash
# gemm_ppw_kernel with B0 read at the end of the previous k-tile: tests, per-shape A/B vs HEAD, stamps, BERT A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/ppwb0; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_ppp_gpu.py tests/test_gemm_gpu.py tests/test_transformer_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ab new; do
  so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
  KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_ppw.py > $O/pw_$v.txt 2>&1 || { tail -20 $O/pw_$v.txt; exit 1; }
done
paste -d'|' $O/pw_ab.txt $O/pw_new.txt | grep ppw | awk -F'|' '{split($1,a," "); split($2,b," "); printf "%-6s %-20s %8s -> %8s us\n", a[1], a[2], a[3], b[3]}'
KFA_KERNELS_SO=_hip_kernels_pw1.so timeout -k 10 180 python3 -u tools/ppw_stamps.py 32768x2304x768 32768x768x3072 > $O/st.txt 2>&1 || { tail -20 $O/st.txt; exit 1; }
grep -v amdgpu.ids $O/st.txt
for i in 1 2 3; do
  for v in ab new; do
    so=_hip_kernels.so; [[ $v == ab ]] && so=_hip_kernels_ab.so
    r=$(KFA_KERNELS_SO=$so timeout -k 10 300 python3 -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 2>$O/bert_$v.err | tail -1) || { tail -20 $O/bert_$v.err; exit 1; }
    echo "bert $v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
