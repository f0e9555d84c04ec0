# PMC passes over tools/bench_attn.py (BERT-base attention fwd / bwd): issue mix and stalls
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_attn/p$i -o p \
    -- python3 $R/tools/bench_attn.py > $R/gpurun_out/pmc_attn/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_attn/p$i.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_attn/p*/*counter_collection.csv'):
    per = collections.defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
        if 'attn' not in k:
            continue
        key = (k, r['Dispatch_Id'], r['Counter_Name'])
        per[key] += float(r['Counter_Value'])
        meta[(k, r['Dispatch_Id'])] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    for (k, d, c), v in per.items():
        vals[k][c].append(v)
    for (k, d), t in meta.items():
        dur[k].append(t)
for k in sorted(vals):
    print(k, 'mean us %.1f' % (sum(dur[k]) / len(dur[k]) / 1e3))
    for c in sorted(vals[k]):
        v = vals[k][c]
        print('   %-28s %.4g' % (c, sum(v) / len(v)))
PY
