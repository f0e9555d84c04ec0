set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gemm_ppp_gpu.py tests/test_attention_gpu.py tests/test_widedeep_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t8.log 2>&1; rc=$?; tail -3 gpurun_out/t8.log; [[ $rc -eq 0 ]] || { tail -30 gpurun_out/t8.log; exit 1; }
bash tools/gpu_r4.sh attn wdb wdown gemm wd profb
