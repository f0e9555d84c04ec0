set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -40 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
timeout -k 10 200 python -u tools/bench_stem.py > gpurun_out/bench_stem_ab.log 2>&1 || { tail -30 gpurun_out/bench_stem_ab.log; exit 1; }
cat gpurun_out/bench_stem_ab.log
for bt in 0 1; do
KFA_BATCHED_TRANSPOSE=$bt timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bt$bt.log 2>&1 || { tail -30 gpurun_out/bench_bt$bt.log; exit 1; }
tail -1 gpurun_out/bench_bt$bt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batched_transpose=$bt', d['value'], d['ms_per_step'])"
done
