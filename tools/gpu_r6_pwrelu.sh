#!/bin/bash
# W&D: the wave-specialised GEMM with the bias + ReLU store epilogue (ppw256-relu) — numerics, in-model re-timing of
# the dense-layer decisions (KFA_ROUTES=retune), merged table vs committed (interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6pwrelu; mkdir -p $O
T=$R/$O/rt.json; rm -f $T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_ppp_gpu.py -k "relu or gelu" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
KFA_ROUTES=retune KFA_ROUTES_DUMP=$T KFA_ROUTES_LOG=1 timeout -k 10 400 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 3 --warmup 2 > $O/rt.log 2> $O/rt.err || { tail -20 $O/rt.err; exit 1; }
grep "dense_fwd" $O/rt.err | cut -c1-300
python - <<PY
import json
base = json.load(open("kubeflow_controller_amd/ops/routes_gfx950.json"))
new = json.load(open("$T"))
n = 0
for k, v in new["routes"].items():
    if k.startswith("dense_fwd|") and "ppw256-relu" in (new["timings_ms"].get(k) or {}):
        base["routes"][k] = v
        base["timings_ms"][k] = new["timings_ms"][k]
        n += 1
json.dump(base, open("$O/merged.json", "w"), indent=1, sort_keys=True)
print("merged", n)
PY
for i in 1 2 3; do
timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > $O/old$i.log 2> $O/old$i.err || { tail -20 $O/old$i.err; exit 1; }
echo "old $(tail -1 $O/old$i.log | cut -c1-140)"
KFA_ROUTES_FILE=$R/$O/merged.json timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 20 --warmup 5 > $O/new$i.log 2> $O/new$i.err || { tail -20 $O/new$i.err; exit 1; }
echo "new $(tail -1 $O/new$i.log | cut -c1-140)"
done
