#!/bin/bash
# BERT FFN-up routed with its bias/GELU pass (GEMM + consumer timed together): in-model
# decision, merged table, interleaved A/B against the committed table with the old
# GEMM-only route (KFA_FFN_UP_PAIR=0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6ffn; mkdir -p $O
T=$R/$O/rt.json; rm -f $T
KFA_ROUTES_DUMP=$T KFA_ROUTES_LOG=1 timeout -k 10 400 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 3 --warmup 2 > $O/rt.log 2> $O/rt.err || { tail -20 $O/rt.err; exit 1; }
grep "ffn_up" $O/rt.err | cut -c1-300
python - <<PY
import json
base = json.load(open("kubeflow_controller_amd/ops/routes_gfx950.json"))
new = json.load(open("$T"))
n = 0
for k, v in new["routes"].items():
    if k.startswith("ffn_up|"):
        base["routes"][k] = v
        base["timings_ms"][k] = new["timings_ms"].get(k)
        n += 1
json.dump(base, open("$O/merged.json", "w"), indent=1, sort_keys=True)
print("merged", n)
PY
for i in 1 2 3; do
KFA_FFN_UP_PAIR=0 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/old$i.log 2> $O/old$i.err || { tail -20 $O/old$i.err; exit 1; }
echo "old $(tail -1 $O/old$i.log | cut -c1-120)"
KFA_ROUTES_FILE=$R/$O/merged.json timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 20 --warmup 5 > $O/new$i.log 2> $O/new$i.err || { tail -20 $O/new$i.err; exit 1; }
echo "new $(tail -1 $O/new$i.log | cut -c1-120)"
done
