#!/bin/bash
# Round-5 evidence: ResNet-50 as a TFJob through the controller (1 worker) and the
# 1-GPU async-PS rehearsal (device transport + collective), after the comm-layer change
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 80 > gpurun_out/r5_tfjob_r50.log 2> gpurun_out/r5_tfjob_r50.err || { tail -20 gpurun_out/r5_tfjob_r50.err; exit 1; }
tail -1 gpurun_out/r5_tfjob_r50.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_ev_bench.log 2> gpurun_out/r5_ev_bench.err || { tail -20 gpurun_out/r5_ev_bench.err; exit 1; }
tail -1 gpurun_out/r5_ev_bench.log
timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device,collective:- > gpurun_out/r5_async_rehearsal.log 2>&1 || { tail -30 gpurun_out/r5_async_rehearsal.log; exit 1; }
tail -15 gpurun_out/r5_async_rehearsal.log
