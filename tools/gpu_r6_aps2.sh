#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6aps2; mkdir -p $O
KFA_PS_SIGNAL_STATS=1 KFA_PS_DEVICE_SIGNAL=1 timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device > $O/reh.log 2>&1 || { tail -20 $O/reh.log; exit 1; }
grep -E 'async' $O/reh.log | tail -1
grep -h "device-signal" gpurun_out/rehearsal_async_device_worker*.log
