set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 200 python -u tools/bench_gemm.py dense > gpurun_out/bench_gemm.log 2>&1 || { tail -30 gpurun_out/bench_gemm.log; exit 1; }
cat gpurun_out/bench_gemm.log
for g in 0 1; do
KFA_GEMM=$g timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 > gpurun_out/bert_gemm$g.log 2>&1 || { tail -30 gpurun_out/bert_gemm$g.log; exit 1; }
echo "KFA_GEMM=$g $(tail -1 gpurun_out/bert_gemm$g.log)"
done
