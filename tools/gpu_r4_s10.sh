# Round-4 session 10: the GPU tests touched since session 9, benches, BERT trace, BERT A/B
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_gemm_gpu.py tests/test_gemm_ppp_gpu.py tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t10.log 2>&1; rc=$?; tail -3 gpurun_out/t10.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/t10.log; exit 1; }
bash tools/gpu_r4.sh bert wdb profb wd abbert
