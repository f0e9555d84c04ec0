#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6ppw192; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ppp_gpu.py -k "ppw192" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/bench_ppw192.py $O/times.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
cut -c1-150 $O/bench.log
