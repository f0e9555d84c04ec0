set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
timeout -k 10 600 python -u tools/tfjob_bench.py examples/tfjob/resnet50-dp8.yml --workers 1 --steps 60 > gpurun_out/tfjob_r50.log 2> gpurun_out/tfjob_r50.err; tail -1 gpurun_out/tfjob_r50.log; tail -5 gpurun_out/tfjob_r50.err
