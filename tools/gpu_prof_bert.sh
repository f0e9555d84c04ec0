#!/bin/bash
# rocprofv3 kernel traces of the BERT-base step with the dense projections on
# hipBLASLt (KFA_GEMM=0) and on the hand-written GEMM (KFA_GEMM=${1:-fused}).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for cfg in 0 ${1:-fused}; do
  KFA_GEMM=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profb_$cfg -o b \
    -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 3 \
    > $R/gpurun_out/profb_$cfg.log 2>&1 || { tail -20 $R/gpurun_out/profb_$cfg.log; exit 1; }
  cd $R
  ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/profb_$cfg.log') if l.startswith('{')][-1]['ms_per_step'])")
  python3 tools/profile_summary.py $(ls gpurun_out/profb_$cfg/*kernel_trace.csv | head -1) 5 "$ms" "BERT-base 256x128 KFA_GEMM=$cfg" adam_kernel > gpurun_out/profb_$cfg.md
  head -45 gpurun_out/profb_$cfg.md
  cd /tmp
done
