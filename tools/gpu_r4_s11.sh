set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t11.log 2>&1; rc=$?; tail -3 gpurun_out/t11.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/t11.log; exit 1; }
bash tools/gpu_r4.sh abbert
