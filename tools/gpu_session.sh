#!/bin/bash
# One gpurun session: GPU tests, the 1-GPU headline bench, a 2-rank gloo
# rehearsal of the multi-GPU launcher on the one GPU, and a rocprofv3 kernel
# trace of the bench (summaries land in gpurun_out/; copy what matters to
# profiles/).  Every GPU step has its own time limit and the chain stops at the
# first failure.
#   gpurun --timeout 900 -- bash tools/gpu_session.sh [tests|bench|prof|all]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
what=${1:-all}
step() { echo "== $(date +%T) $*" | tee -a gpurun_out/session.log; }

if [[ $what == tests || $what == all ]]; then
  step "pytest -m gpu"
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
if [[ $what == bench || $what == all ]]; then
  step "bench 1 GPU"
  KFA_CONV_TUNE_LOG=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 \
    > gpurun_out/bench1.log 2> gpurun_out/bench1.err || { tail -30 gpurun_out/bench1.err; exit 1; }
  tail -1 gpurun_out/bench1.log
  step "bench 1 GPU, whole step as one HIP graph"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph on \
    > gpurun_out/bench1_graph.log 2> gpurun_out/bench1_graph.err || { tail -30 gpurun_out/bench1_graph.err; exit 1; }
  tail -1 gpurun_out/bench1_graph.log
  step "bench --gpus 2 (gloo rehearsal on one GPU)"
  KFA_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 \
    > gpurun_out/bench2_gloo.log 2> gpurun_out/bench2_gloo.err || { tail -30 gpurun_out/bench2_gloo.err; exit 1; }
  tail -1 gpurun_out/bench2_gloo.log
fi
if [[ $what == prof || $what == all ]]; then
  step "rocprofv3 kernel trace of bench"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o r50 \
    -- python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  cd "$R"
  f=$(ls gpurun_out/prof/*kernel_trace.csv 2>/dev/null | head -1)
  ms=$(python3 -c "import json,sys;print([json.loads(l) for l in open('gpurun_out/prof.log') if l.startswith('{')][-1]['ms_per_step'])")
  python3 tools/profile_summary.py "$f" 10 "$ms" "ResNet-50 bs256 1x MI355X (HEAD)" > gpurun_out/prof_summary.md
  head -40 gpurun_out/prof_summary.md
fi
step done
