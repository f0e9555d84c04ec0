set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -60 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
for S in 128 512; do
B=$((256 * 128 / S))
timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch $B --seq $S > gpurun_out/bert_s$S.log 2>&1 || { tail -30 gpurun_out/bert_s$S.log; exit 1; }
echo "S=$S B=$B $(tail -1 gpurun_out/bert_s$S.log)"
done
KFA_FUSED_ATTN=0 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 64 --seq 512 > gpurun_out/bert_s512_split.log 2>&1 || { tail -30 gpurun_out/bert_s512_split.log; exit 1; }
echo "split S=512 $(tail -1 gpurun_out/bert_s512_split.log)"
