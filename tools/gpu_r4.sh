#!/bin/bash
# Round-4 GPU session: GPU tests, the headline bench, BERT-base / Wide&Deep benches
# (per-shape GEMM tuner log), a Wide&Deep kernel trace, an env A/B, PMC passes.
# Each GPU step has its own time limit; the chain stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_r4.sh [steps...]   (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
steps=${*:-"tests bench bert wd abm pmc"}
log() { echo "== $(date +%T) $*" | tee -a gpurun_out/r4_session.log; }
for s in $steps; do
  case $s in
    tests)
      log "pytest -m gpu"
      # a failing test does not stop the session (perf numbers still wanted), a GPU fault / hang does
      timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests.log 2>&1
      rc=$?
      tail -3 gpurun_out/gpu_tests.log
      if [[ $rc -ne 0 ]]; then
        tail -40 gpurun_out/gpu_tests.log
        if [[ $rc -ge 124 ]] || grep -qiE "illegal memory|memory access fault|hardware exception|GPU Hang|Timeout \(0:" gpurun_out/gpu_tests.log; then
          echo "GPU fault / hang in the tests: stopping"; exit 1
        fi
        echo "TESTS FAILED (rc $rc): continuing with the measurements"
      fi ;;
    bench)
      log "bench 1 GPU"
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2> gpurun_out/bench1.err \
        || { tail -30 gpurun_out/bench1.err; exit 1; }
      tail -1 gpurun_out/bench1.log ;;
    bert)
      log "BERT-base 256x128"
      KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 --seq 128 \
        --steps 20 --warmup 5 > gpurun_out/bert.log 2> gpurun_out/bert.err || { tail -30 gpurun_out/bert.err; exit 1; }
      tail -1 gpurun_out/bert.log; grep "kfa gemm tune" gpurun_out/bert.err | head -20 ;;
    wd)
      log "Wide&Deep kernel trace"
      KFA_GEMM_TUNE_LOG=1 bash tools/gpu_prof_wd.sh 2> gpurun_out/wd_tune.err || exit 1 ;;
    wdb)
      log "Wide&Deep bench (unprofiled)"
      timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 --steps 30 --warmup 5 \
        > gpurun_out/wdb.log 2> gpurun_out/wdb.err || { tail -30 gpurun_out/wdb.err; exit 1; }
      tail -1 gpurun_out/wdb.log ;;
    wdown)
      log "Wide&Deep bench, own GEMMs on every covered shape (KFA_GEMM=own)"
      KFA_GEMM=own KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model wide_deep --batch 65536 \
        --steps 30 --warmup 5 > gpurun_out/wdown.log 2> gpurun_out/wdown.err || { tail -30 gpurun_out/wdown.err; exit 1; }
      tail -1 gpurun_out/wdown.log; grep "kfa gemm tune" gpurun_out/wdown.err | head -10 ;;
    bertown)
      log "BERT-base 256x128, own GEMMs on every covered shape (KFA_GEMM=own)"
      KFA_GEMM=own KFA_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u tools/bench_model.py --model bert_base --batch 256 \
        --seq 128 --steps 20 --warmup 5 > gpurun_out/bertown.log 2> gpurun_out/bertown.err \
        || { tail -30 gpurun_out/bertown.err; exit 1; }
      tail -1 gpurun_out/bertown.log; grep "kfa gemm tune" gpurun_out/bertown.err | head -20 ;;
    attn)
      log "attention S=128: bwd D through LDS (PF=1) vs global scratch (PF=0)"
      for v in 0 1 0 1; do
        KFA_ATTN_PF=$v timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | tee -a gpurun_out/attn.log | grep "attn PF" || exit 1
      done ;;
    stagger)
      log "GEMM C-burst stagger sweep"
      KFA_PPP_STAGGER=1 timeout -k 10 300 python -u tools/bench_ppp.py > gpurun_out/stagger.log 2>&1 \
        || { tail -20 gpurun_out/stagger.log; exit 1; }
      cat gpurun_out/stagger.log ;;
    ab)
      log "A/B conv wgrad side stream"
      bash tools/gpu_ab_env.sh "KFA_CONV_WGRAD_SIDE=0" "KFA_CONV_WGRAD_SIDE=1 KFA_CONV_OVERSUB=2" || exit 1 ;;
    abm)
      log "A/B/C... ResNet-50 knobs"
      AB_ROUNDS=2 bash tools/gpu_ab_multi.sh "BASE=1" "KFA_CONV_WGRAD_SIDE=1 KFA_CONV_OVERSUB=2" \
        "KFA_WGRAD_WIDE64_ANY=1" "KFA_CONV_NARROW_LONGK=3" "KFA_CONV_BIG_AUTO_E=0" "KFA_POOL_BN_STATS=0 KFA_POOL_BWD4=0" \
        | tee gpurun_out/abm.log || exit 1 ;;
    async)
      log "async PS rehearsal (device transport), BERT-base 2w+1ps on one GPU"
      timeout -k 10 400 python -u tools/async_rehearsal.py --modes async:device,collective:- 2>&1 \
        | tee gpurun_out/async_rehearsal.log || exit 1 ;;
    profb)
      log "BERT-base kernel trace (HEAD)"
      bash tools/gpu_prof_bert_head.sh || exit 1 ;;
    abbert)
      log "A/B/C BERT-base knobs"
      AB_ROUNDS=2 AB_CMD="tools/bench_model.py --model bert_base --batch 256 --seq 128" bash tools/gpu_ab_multi.sh \
        "BASE=1" "KFA_FFN_GELU_EPI=0" | tee gpurun_out/abbert.log || exit 1 ;;
    abwd)
      log "A/B/C Wide&Deep knobs"
      AB_ROUNDS=2 AB_CMD="tools/bench_model.py --model wide_deep --batch 65536" bash tools/gpu_ab_multi.sh \
        "BASE=1" "KFA_WGRAD_MIN_STEPS=16" "KFA_WGRAD_MIN_STEPS=32" "KFA_WGRAD_MIN_STEPS=64" \
        | tee gpurun_out/abwd.log || exit 1 ;;
    gemm)
      log "GEMM shapes: hipBLASLt vs own"
      timeout -k 10 300 python -u tools/bench_ppp.py > gpurun_out/bench_ppp.log 2>&1 || { tail -20 gpurun_out/bench_ppp.log; exit 1; }
      cat gpurun_out/bench_ppp.log ;;
    pmc)
      log "PMC round-3 kernels"
      bash tools/gpu_pmc_r4.sh > gpurun_out/pmc_r4.log 2>&1 || { tail -20 gpurun_out/pmc_r4.log; exit 1; }
      head -60 gpurun_out/pmc_r4/table.txt ;;
  esac
done
log done
