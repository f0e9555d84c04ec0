set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -40 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
for v in 1 3; do
echo "== narrow variant $v"
KFA_CONV_NARROW=$v timeout -k 10 200 python -u tools/bench_stem.py > gpurun_out/bench_stem_v$v.log 2>&1 || { tail -30 gpurun_out/bench_stem_v$v.log; exit 1; }
grep ours_fwd gpurun_out/bench_stem_v$v.log
KFA_CONV_NARROW=$v timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/bench_conv_v$v.log 2>&1 || { tail -30 gpurun_out/bench_conv_v$v.log; exit 1; }
grep "Cout   64\|TOTAL" gpurun_out/bench_conv_v$v.log
done
