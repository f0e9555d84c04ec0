#!/bin/bash
# W&D: which step phase issues the runtime copy kernel (__amd_rocclr_copyBuffer): kernel-trace
# neighbours of each copy in one step, plus a torch.profiler op table for aten::copy_ callers
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6wdc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/wt -o w \
  -- python3 $R/tools/bench_model.py --model wide_deep --batch 65536 --steps 4 --warmup 3 > $R/$O/wd_trace.log 2>&1 || { tail -20 $R/$O/wd_trace.log; exit 1; }
cd $R
python3 - <<'PY' > $O/neighbours.txt
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r6wdc/wt/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void (anonymous namespace)::adam_kernel<true>")]
a, b = ad[-2], ad[-1]
for r in rows[a:b + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{d:8.1f} us  q{r.get('Queue_Id','')} s{r.get('Stream_Id','')}  {r['Kernel_Name'][:110]}")
PY
rm -f $O/wt/*kernel_trace.csv
cat $O/neighbours.txt
