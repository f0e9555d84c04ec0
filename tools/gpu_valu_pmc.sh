# One PMC pass (issue mix) over the ResNet-50 and BERT-base steps: VALU / SALU / MFMA / LDS
# instructions and VALU-active cycles per kernel -> gpurun_out/valu_{r50,bert}.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/valu
cd /tmp && export TMPDIR=/tmp
SET="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d $R/gpurun_out/valu/r50 -o p \
  -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/valu/r50.log 2>&1 || { tail -5 $R/gpurun_out/valu/r50.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d $R/gpurun_out/valu/bert -o p \
  -- python3 $R/tools/bench_model.py --model bert_base --batch 256 --seq 128 --steps 2 --warmup 2 > $R/gpurun_out/valu/bert.log 2>&1 || { tail -5 $R/gpurun_out/valu/bert.log; exit 1; }
cd $R
python3 tools/valu_table.py gpurun_out/valu/r50/p_counter_collection.csv > gpurun_out/valu_r50.md
python3 tools/valu_table.py gpurun_out/valu/bert/p_counter_collection.csv > gpurun_out/valu_bert.md
head -25 gpurun_out/valu_r50.md; head -25 gpurun_out/valu_bert.md
