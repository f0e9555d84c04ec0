#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6lp; mkdir -p $O
timeout -k 10 300 python -u tools/launch_profile.py --model resnet50 > $O/r50_launches.txt 2> $O/r50.err || { tail -20 $O/r50.err; exit 1; }
tail -30 $O/r50_launches.txt
