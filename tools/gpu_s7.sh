set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_async_ps_gpu.py -x -q --timeout 150 --timeout-method thread -k replica > gpurun_out/async_tests.log 2>&1 || { tail -80 gpurun_out/async_tests.log; exit 1; }
tail -4 gpurun_out/async_tests.log
