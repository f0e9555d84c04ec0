#!/bin/bash
# New-feature checks first (graph replay, 64x256 wgrad), then the full GPU suite,
# then same-box A/Bs (wgrad tile, HIP graph, conv MFMA-phase priority) and a kernel trace.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_conv_gpu.py -k "graph or wgrad" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { tail -40 gpurun_out/new_tests.log; exit 1; }
tail -3 gpurun_out/new_tests.log
bash tools/gpu_session.sh tests || exit 1
echo "== A/B wgrad 64x256"
bash tools/gpu_ab_env.sh KFA_WGRAD_WIDE64=0 KFA_WGRAD_WIDE64=1 || exit 1
echo "== A/B HIP graph"
bash tools/gpu_ab_env.sh KFA_GRAPH=off KFA_GRAPH=on || exit 1
echo "== A/B conv setprio (A = default build, B = _hip_kernels_prio.so)"
bash tools/gpu_ab_env.sh KFA_KERNELS_SO=_hip_kernels.so KFA_KERNELS_SO=_hip_kernels_prio.so || exit 1
bash tools/gpu_session.sh prof || exit 1
