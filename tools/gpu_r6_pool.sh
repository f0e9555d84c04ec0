#!/bin/bash
# stem BN + ReLU + max pool forward without per-tap bf16 rounding: pool tests, then a short
# ResNet-50 kernel trace (the pool kernels' per-step time)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6pool; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pool" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rt -o r -- python3 $R/bench.py --steps 10 --warmup 5 > $R/$O/r50.log 2>&1 || { tail -20 $R/$O/r50.log; exit 1; }
cd $R
grep -i "maxpool" $O/rt/r_kernel_stats.csv | cut -d, -f1-6
grep '^{' $O/r50.log | cut -c1-200
rm -f $O/rt/*kernel_trace.csv
