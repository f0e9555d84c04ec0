#!/bin/bash
# 256x64 vs 128x64 conv tiles for the N <= 64 launches: in-model re-timing of every conv
# decision (KFA_ROUTES=retune), the N <= 64 picks merged into the committed table, then
# ResNet-50 on the committed table vs the merged one (interleaved)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6narrow; mkdir -p $O
T=$R/$O/rt.json; rm -f $T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
KFA_ROUTES=retune KFA_ROUTES_DUMP=$T KFA_ROUTES_LOG=1 timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 > $O/rt.log 2> $O/rt.err || { tail -20 $O/rt.err; exit 1; }
grep "igemm256x64\|igemm128x64" $O/rt.err | cut -c1-260
python - <<PY
import json
base = json.load(open("kubeflow_controller_amd/ops/routes_gfx950.json"))
new = json.load(open("$T"))
n = 0
for k, v in new["routes"].items():
    t = new["timings_ms"].get(k) or {}
    if "igemm256x64" in t or "igemm128x64" in t:
        base["routes"][k] = v
        base["timings_ms"][k] = t
        n += 1
json.dump(base, open("$O/merged.json", "w"), indent=1, sort_keys=True)
print("merged", n)
PY
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/old$i.log 2> $O/old$i.err || { tail -20 $O/old$i.err; exit 1; }
echo "old $(tail -1 $O/old$i.log | cut -c1-130)"
KFA_ROUTES_FILE=$R/$O/merged.json timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/new$i.log 2> $O/new$i.err || { tail -20 $O/new$i.err; exit 1; }
echo "new $(tail -1 $O/new$i.log | cut -c1-130)"
done
