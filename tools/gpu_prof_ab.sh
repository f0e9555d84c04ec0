#!/bin/bash
# Kernel traces of the ResNet-50 bench under two settings of one env var:
#   gpurun -- bash tools/gpu_prof_ab.sh VAR VAL_A VAL_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
var=$1; shift
for val in "$@"; do
  cd /tmp && export TMPDIR=/tmp
  export $var=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_$val -o r \
    -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/pab_$val.log 2>&1 || { tail -20 $R/gpurun_out/pab_$val.log; exit 1; }
  cd $R
  ms=$(python3 -c "import json;print([json.loads(l) for l in open('gpurun_out/pab_$val.log') if l.startswith('{')][-1]['ms_per_step'])")
  python3 tools/profile_summary.py $(ls gpurun_out/pab_$val/*kernel_trace.csv | head -1) 10 "$ms" "ResNet-50 $var=$val" > gpurun_out/pab_$val.md
done
