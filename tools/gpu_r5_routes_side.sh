#!/bin/bash
# routing table regeneration (igemm128 candidate added), then the conv-wgrad side-stream A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
bash tools/gpu_r5_routes.sh || exit 1
export KFA_ROUTES_FILE=$(pwd)/gpurun_out/routes_gfx950.json
bash tools/gpu_ab_env.sh "KFA_SIDE_STREAM=0" "KFA_SIDE_STREAM=1 KFA_CONV_WGRAD_SIDE=1"
