#!/bin/bash
# PMC pass over BERT-base GEMM dispatches (ppw3 + hipBLASLt), FFN-down forward forced onto ppw192
# (p3072) and the committed table (base): L2 hit/miss and HBM request counts per dispatch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6pmc; mkdir -p $O
export TMPDIR=/tmp
for v in p3072 base; do
  f=$R/kubeflow_controller_amd/ops/routes_gfx950.json; [ $v != base ] && f=$R/tools/routes_ab/$v.json
  KFA_ROUTES_FILE=$f timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --kernel-include-regex 'ppw3|Cijk' --output-format csv -d $O/$v -o p -- \
    python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 2 --warmup 2 > $O/$v.log 2> $O/$v.err || exit 1
done
