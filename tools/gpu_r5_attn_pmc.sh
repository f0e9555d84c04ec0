#!/bin/bash
# Round-5 attention PMC table: four passes over tools/bench_attn.py (BERT-base 256 x 128,
# 12 heads, p = 0.1; every fwd / bwd form of the bench line), then the BERT step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/pmc_attn5
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_attn5/p$i -o p \
    -- python3 $R/tools/bench_attn.py > $R/gpurun_out/pmc_attn5/p$i.log 2>&1 || { tail -5 $R/gpurun_out/pmc_attn5/p$i.log; exit 1; }
done
cd $R
python3 tools/pmc_derived.py $(ls gpurun_out/pmc_attn5/p*/*counter_collection.csv) > gpurun_out/pmc_attn5/derived.md
python3 tools/pmc_derived.py --issue $(ls gpurun_out/pmc_attn5/p*/*counter_collection.csv) > gpurun_out/pmc_attn5/issue.md
cat gpurun_out/pmc_attn5/derived.md gpurun_out/pmc_attn5/issue.md
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 10 --warmup 3 > gpurun_out/r5_attn_bert2.log 2> gpurun_out/r5_attn_bert2.err || { tail -20 gpurun_out/r5_attn_bert2.err; exit 1; }
tail -1 gpurun_out/r5_attn_bert2.log
