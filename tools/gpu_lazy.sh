set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_e2e_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lazy_t.log 2>&1; rc=$?; tail -3 gpurun_out/lazy_t.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/lazy_t.log; exit 1; }
AB_ROUNDS=3 bash tools/gpu_ab_multi.sh "BASE=1" "KFA_LAZY_BN2=0" | tee gpurun_out/ab_lazy.log
