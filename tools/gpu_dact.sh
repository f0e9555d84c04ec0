set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_ppp_gpu.py -x -q --timeout 120 --timeout-method thread -k "gelu_backward" > gpurun_out/dact_t.log 2>&1; rc=$?; tail -5 gpurun_out/dact_t.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/dact_t.log; exit 1; }
timeout -k 10 300 python -u tools/bench_dact.py 2>&1 | tee gpurun_out/dact_b.log
