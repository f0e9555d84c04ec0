#!/bin/bash
# Round-6 check as the driver runs it: every GPU test, smoke(), the 1-GPU bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 1; }
tail -1 gpurun_out/bench1.log
