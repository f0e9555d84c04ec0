# Sparse-update session: the sort/segment tests, the radix micro-bench, then the
# W&D kernel trace (tools/gpu_r4.sh wd).  Extra steps of gpu_r4.sh as arguments.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sparse_gpu.py tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sparse_tests.log 2>&1; rc=$?; tail -5 gpurun_out/sparse_tests.log
[[ $rc -eq 0 ]] || exit 1
PYTHONPATH=. timeout -k 10 120 python -u tools/bench_radix.py 2>&1 | tee gpurun_out/bench_radix.log || exit 1
bash tools/gpu_r4.sh wd "$@"
