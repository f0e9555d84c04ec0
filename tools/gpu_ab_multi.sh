#!/bin/bash
# Same-box A/B/C/... of the ResNet-50 step over several environment settings,
# interleaved (R rounds, default 2):
#   gpurun -- bash tools/gpu_ab_multi.sh "BASE=1" "KFA_X=1" "KFA_Y=1 KFA_Z=0" ...
# "BASE=1" (any unused variable) is the unmodified default.  One line per run:
# <variant index> (<env>) <images/s> <ms/step>.  AB_CMD overrides the benchmark
# (e.g. AB_CMD="tools/bench_model.py --model bert_base --batch 256 --seq 128").
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
R=${AB_ROUNDS:-2}
for i in $(seq 1 $R); do
  v=0
  for e in "$@"; do
    r=$(env $e timeout -k 10 240 python -u ${AB_CMD:-bench.py} --steps 20 --warmup 5 2>gpurun_out/abm_$v.err | tail -1) \
      || { tail -20 gpurun_out/abm_$v.err; exit 1; }
    echo "$v ($e) $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
    v=$((v+1))
  done
done
