#!/bin/bash
# Same-box A/B of the ResNet-50 step: ops/$ABSO (A) vs ops/_hip_kernels.so (B), interleaved, 3 rounds.
#   gpurun -- env ABSO=_hip_kernels_nh2.so bash tools/gpu_ab_so.sh [bench args]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [[ $v == A ]]; then so=${ABSO:-_hip_kernels_ab.so}; else so=_hip_kernels.so; fi
    r=$(KFA_KERNELS_SO=$so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" 2>gpurun_out/ab_$v.err | tail -1) \
      || { tail -20 gpurun_out/ab_$v.err; exit 1; }
    echo "$v $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
