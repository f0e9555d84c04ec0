#!/bin/bash
# round-6: comm / overlap / DP GPU tests + world-1 bench JSON fields
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/r6comm; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_opt_overlap_gpu.py tests/test_dp_gpu.py tests/test_comm_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|overlap adam" $O/tests.log | tail -5
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/r50.log 2> $O/r50.err || { tail -20 $O/r50.err; exit 1; }
tail -1 $O/r50.log
