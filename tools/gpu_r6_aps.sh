#!/bin/bash
# async PS: device-side IPC-event hand-offs vs host waits — GPU tests, BERT-base rehearsal A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6aps; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_async_ps_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -12
for i in 1 2; do
for s in 1 0; do
KFA_PS_DEVICE_SIGNAL=$s timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device > $O/reh_$s$i.log 2>&1 || { tail -20 $O/reh_$s$i.log; exit 1; }
echo "signal=$s $(grep -E 'async' $O/reh_$s$i.log | tail -1)"
done
done
