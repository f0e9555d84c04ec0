#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/aten
timeout -k 10 300 python3 -u tools/aten_in_step.py bert > gpurun_out/aten/bert.txt 2>&1 || { tail -20 gpurun_out/aten/bert.txt; exit 1; }
cat gpurun_out/aten/bert.txt | grep "us/step"
timeout -k 10 300 python3 -u tools/aten_in_step.py resnet > gpurun_out/aten/r50.txt 2>&1 || { tail -20 gpurun_out/aten/r50.txt; exit 1; }
cat gpurun_out/aten/r50.txt | grep "us/step"
