#!/bin/bash
# Regenerate the committed routing table (ops/routes_gfx950.json) by timing every
# per-shape decision of the three headline steps (ResNet-50, BERT-base, W&D), then
# run the ResNet bench on the table.  KFA_ROUTES=retune: ignore the old table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
rocm-smi --showclocks > gpurun_out/r5_routes_clocks.log 2>&1 || true
T=gpurun_out/routes_gfx950.json; rm -f $T
export KFA_ROUTES=retune KFA_ROUTES_DUMP=$R/$T KFA_ROUTES_LOG=1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r5_rt_r50.log 2> gpurun_out/r5_rt_r50.err || { tail -20 gpurun_out/r5_rt_r50.err; exit 1; }
tail -1 gpurun_out/r5_rt_r50.log
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 2 > gpurun_out/r5_rt_bert.log 2> gpurun_out/r5_rt_bert.err || { tail -20 gpurun_out/r5_rt_bert.err; exit 1; }
tail -1 gpurun_out/r5_rt_bert.log
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 10 --warmup 3 > gpurun_out/r5_rt_wd.log 2> gpurun_out/r5_rt_wd.err || { tail -20 gpurun_out/r5_rt_wd.err; exit 1; }
tail -1 gpurun_out/r5_rt_wd.log
unset KFA_ROUTES KFA_ROUTES_DUMP KFA_ROUTES_LOG
export KFA_ROUTES_FILE=$R/$T
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_rt_b$i.log 2> gpurun_out/r5_rt_b$i.err || { tail -20 gpurun_out/r5_rt_b$i.err; exit 1; }
tail -1 gpurun_out/r5_rt_b$i.log
done
KFA_CONV_PP=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_rt_nopp.log 2> gpurun_out/r5_rt_nopp.err || { tail -20 gpurun_out/r5_rt_nopp.err; exit 1; }
tail -1 gpurun_out/r5_rt_nopp.log
