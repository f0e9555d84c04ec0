#!/bin/bash
# BERT-base in-model GEMM timings with the ppw192 candidates (KFA_ROUTES=retune), then
# BERT-base on the committed table vs the table with the re-timed proj / proj_dgrad picks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6bert; mkdir -p $O
T=$R/$O/bert_routes.json; rm -f $T
KFA_ROUTES=retune KFA_ROUTES_DUMP=$T KFA_ROUTES_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 5 --warmup 2 > $O/rt.log 2> $O/rt.err || { tail -20 $O/rt.err; exit 1; }
grep -E "proj|dense_fwd|decoder" $O/rt.err | cut -c1-300
python - <<PY
import json
base = json.load(open("kubeflow_controller_amd/ops/routes_gfx950.json"))
new = json.load(open("$T"))
for k, v in new["routes"].items():
    if k.startswith(("proj|", "proj_dgrad|")):
        base["routes"][k] = v
        base["timings_ms"][k] = new["timings_ms"].get(k, base["timings_ms"].get(k))
json.dump(base, open("$O/merged.json", "w"), indent=1, sort_keys=True)
PY
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/old$i.log 2> $O/old$i.err || { tail -20 $O/old$i.err; exit 1; }
echo "old $(tail -1 $O/old$i.log | cut -c1-130)"
KFA_ROUTES_FILE=$R/$O/merged.json timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/new$i.log 2> $O/new$i.err || { tail -20 $O/new$i.err; exit 1; }
echo "new $(tail -1 $O/new$i.log | cut -c1-130)"
done
