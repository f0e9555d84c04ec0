#!/bin/bash
# Async PS request channel on the first-party host transport: GPU async-PS tests and the
# 1-GPU BERT async rehearsal (device transport + collective), native vs gloo channel
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_async_ps_gpu.py tests/test_comm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_p2p_tests.log 2>&1; rc=$?
tail -1 gpurun_out/r5_p2p_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/r5_p2p_tests.log; exit 1; }
timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device > gpurun_out/r5_p2p_reh_native.log 2>&1 || { tail -30 gpurun_out/r5_p2p_reh_native.log; exit 1; }
echo "native:"; tail -4 gpurun_out/r5_p2p_reh_native.log
KFA_PS_P2P=torch timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device > gpurun_out/r5_p2p_reh_gloo.log 2>&1 || { tail -30 gpurun_out/r5_p2p_reh_gloo.log; exit 1; }
echo "gloo:"; tail -4 gpurun_out/r5_p2p_reh_gloo.log
