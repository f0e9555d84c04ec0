#!/bin/bash
# gradient-bucket readiness on every model family's HIP path + the distributed GPU tests
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out/ready; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_opt_overlap_gpu.py -x -v --timeout 240 --timeout-method thread > $O/test.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/test.log | tail -12; [[ $rc -eq 0 ]] || { tail -40 $O/test.log; exit 1; }
