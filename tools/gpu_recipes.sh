# The GPU runs of this repository as named recipes over ONE step runner (tools/gpu_steps.sh: each
# step under its own time limit, a normal failure continues, a fault / abort / time limit stops).
#   /usr/local/graft/bin/gpurun --timeout 1500 -- 'bash tools/gpu_recipes.sh <recipe> [<recipe> ...]'
# Outputs: gpurun_out/<step>.log (+ rocprof directories); summaries go to profiles/ by hand
# (tools/summarize_profile.py, tools/pmc_summary.py).
#
#   tests      every GPU test (pytest -m gpu)
#   bench      the headline bench.py (driver's 20/5) + 8 bf16 / 32 fp8 concurrent sessions
#   prof       rocprofv3 kernel trace of a short headline bench
#   pmc        hardware counters: the hot kernels (pmc_kernels.py), the fp8 decode step
#              (pmc_fp8_chain.py) and the Llama-3-70B chained layer (pmc_chain.py)
#   llama70b   config 4 at TP=1 (bench.py --llm llama3-70b) + its kernel trace
#   tp         tools/tp_check.py: TP=2 (small), TP=2/4/8 with Llama-3-70B per-rank shapes, ranks
#              sharing the one GPU (gloo control plane)
#   rows       decode step vs rows per step + batched admission prefill (tools/rows_sweep.py)
#   service    speech end -> intent through the services (tools/service_bench.py)
#   service6   the same with paused speech, end-of-packet timing, commit windows 0 / 700 ms, chain gate
#   asr        Whisper-tiny / large-v3 decode timing + kernel trace (tools/asr_timing.py)
#   frontend   ASR front-end kernel bench + counters (tools/bench_frontend.py, pmc_frontend.py)
TPR="python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1"
PT="python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu"
PMC1="--pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY"
PMC2="--pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
PMC3="--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
KT="--kernel-trace --output-format csv"
steps=()
add() { steps+=("$1" "$2" "$3"); }
pmc3() {  # three counter passes of one target program
  add "$1_p1" 120 "rocprofv3 $PMC1 $KT -d gpurun_out/$1/p1 -- python3 -u $2"
  add "$1_p2" 120 "rocprofv3 $PMC2 $KT -d gpurun_out/$1/p2 -- python3 -u $2"
  add "$1_p3" 120 "rocprofv3 $PMC3 $KT -d gpurun_out/$1/p3 -- python3 -u $2"
}
for r in "$@"; do
  case "$r" in
    tests) add gpu_tests 1200 "$PT tests" ;;
    bench)
      add bench_bf16 400 "python -u bench.py"
      add bench_bf16_c8 500 "python -u bench.py --concurrent 8 --steps 10 --warmup 3"
      add bench_fp8_c32 600 "python -u bench.py --dtype fp8 --concurrent 32 --steps 10 --warmup 3" ;;
    prof) add prof_bf16 400 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 -u bench.py --steps 5 --warmup 2" ;;
    pmc)
      pmc3 pmc_kernels tools/pmc_kernels.py
      pmc3 pmc_fp8 tools/pmc_fp8_chain.py
      pmc3 pmc_chain70 "tools/pmc_chain.py --model llama3-70b --layers 3" ;;
    llama70b)
      add bench_70b 600 "python -u bench.py --llm llama3-70b --steps 5 --warmup 2"
      add prof_chain70 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chain70 -o run -- python3 -u tools/pmc_chain.py --model llama3-70b --layers 3" ;;
    tp)
      add tp2_small 400 "$TPR --nproc-per-node=2 --master-port=29561 tools/tp_check.py"
      for n in 2 4 8; do
        add "tp${n}_70b" 500 "VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=$n --master-port=2957$n tools/tp_check.py"
      done ;;
    rows) add rows_sweep 400 "python -u tools/rows_sweep.py --json gpurun_out/rows_sweep.jsonl" ;;
    service) add service_bench 1100 "python -u tools/service_bench.py --json gpurun_out/service_bench.jsonl" ;;
    service6)  # round 6: paused speech, end-of-packet timing, commit window, chain gated on the ASR
      add svc_tiny 1100 "python -u tools/service_bench.py --sessions 1,8 --debounce 0 --commit 0,700 --chain gate --utterances 16 --json gpurun_out/svc_tiny.jsonl"
      add svc_tiny_par 600 "python -u tools/service_bench.py --sessions 1 --debounce 1000 --commit 0 --chain gate --utterances 12 --json gpurun_out/svc_tiny.jsonl"
      add svc_tiny_pk 600 "python -u tools/service_bench.py --sessions 1 --debounce 0 --commit 0 --chain 0 --utterances 12 --json gpurun_out/svc_tiny.jsonl"
      add svc_large 1100 "python -u tools/service_bench.py --asr whisper-large-v3 --sessions 1,8 --debounce 0 --commit 0,700 --chain gate --utterances 16 --json gpurun_out/svc_large.jsonl" ;;
    asr)
      add asr_tiny 200 "python -u tools/asr_timing.py --asr whisper-tiny"
      add asr_large 300 "python -u tools/asr_timing.py --asr whisper-large-v3 --reps 5"
      add asr_large_prof 400 "rocprofv3 --kernel-trace --stats -d gpurun_out/asr_large_prof -o run -- python3 -u tools/asr_timing.py --asr whisper-large-v3 --reps 3" ;;
    frontend)
      add frontend_bench 300 "python -u tools/bench_frontend.py"
      pmc3 pmc_frontend tools/pmc_frontend.py ;;
    *) echo "unknown recipe $r" >&2; exit 2 ;;
  esac
done
bash "$(dirname "$0")/gpu_steps.sh" "${steps[@]}"
