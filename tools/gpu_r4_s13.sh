set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_ppp_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1; rc=$?; tail -3 gpurun_out/t13.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/t13.log; exit 1; }
bash tools/gpu_r4.sh bert abbert
