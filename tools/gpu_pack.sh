set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [[ $rc -eq 0 ]] || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2> gpurun_out/bench1.err | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 2> gpurun_out/bert.err | tail -1
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 2> gpurun_out/wd.err | tail -1
