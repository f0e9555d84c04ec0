set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_async_ps_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/async_tests.log 2>&1 || { tail -60 gpurun_out/async_tests.log; exit 1; }
tail -4 gpurun_out/async_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
