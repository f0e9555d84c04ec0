#!/bin/bash
# in-step per-call durations of the N = 768 dgrad GEMMs: round-5 table (hipBLASLt) vs HEAD (ppw192)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r6bcalls; mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
for v in r5 head; do
  f=$R/kubeflow_controller_amd/ops/routes_gfx950.json; [ $v = r5 ] && f=$R/kubeflow_controller_amd/ops/routes_gfx950_r5.json
  KFA_ROUTES_FILE=$f timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/$v -o b \
    -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 > $R/$O/$v.log 2>&1 || { tail -20 $R/$O/$v.log; exit 1; }
done
cd $R
for v in r5 head; do
  echo "#### $v"
  python3 tools/trace_calls.py $(ls $O/$v/*kernel_trace.csv | head -1) 4 adam_kernel Cijk_Ailk gemm_ppw3 weight_transpose_multi ln_bwd_kernel attn_bwd bias_act_bwd wgrad_pp Cijk_Alik Custom_Cijk
  rm -f $O/$v/*kernel_trace.csv
done
