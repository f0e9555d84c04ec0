set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -40 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r$i.log 2>&1 || { tail -30 gpurun_out/bench_r$i.log; exit 1; }
echo "run $i $(tail -1 gpurun_out/bench_r$i.log | cut -c1-200)"
done
