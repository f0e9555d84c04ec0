#!/bin/bash
# BN in-kernel finalize retest (tests + ResNet A/B) and the BERT bias_act_bwd
# column-lane A/B (KFA_BIAS_ACT_CL16).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k bn \
  > gpurun_out/kern_tests.log 2>&1 || { tail -30 gpurun_out/kern_tests.log; exit 1; }
tail -1 gpurun_out/kern_tests.log
bash tools/gpu_ab_env.sh "KFA_BN_FOLD=0" "KFA_BN_FOLD=1" && bash tools/gpu_ab_bert.sh "KFA_BIAS_ACT_CL16=0" "KFA_BIAS_ACT_CL16=1"
