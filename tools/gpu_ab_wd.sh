set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 200 python -u -m pytest tests/test_widedeep_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for i in 1 2 3; do for f in 0 1; do
  r=$(KFA_WD_FUSED_INPUT=$f timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 1
  echo "W&D fused_input=$f $(echo "$r" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
