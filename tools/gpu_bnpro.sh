set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn_apply_prologue" > gpurun_out/bnpro_t.log 2>&1; rc=$?; tail -5 gpurun_out/bnpro_t.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/bnpro_t.log; exit 1; }
timeout -k 10 300 python -u tools/bench_bnpro.py 2>&1 | tee gpurun_out/bnpro_b.log
