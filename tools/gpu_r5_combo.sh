#!/bin/bash
# pp / pp128 numerics + per-layer A/B, then the routing-table regeneration + benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
bash tools/gpu_r5_pp.sh || exit 1
bash tools/gpu_r5_routes.sh
