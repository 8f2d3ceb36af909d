set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "handoff or one_launch or tiled_mfma or 8phase or fp8 or qkv or gemm or shared_prefix" > gpurun_out/kt.log 2>&1
timeout -k 10 300 python -u tools/attn_probe.py --impls mq --split-sweep --only-llama > gpurun_out/attn_sweep.log 2>&1
for nb in 4 2; do
  VWA_GEMM_NB=$nb timeout -k 10 300 python -u tools/rows_sweep.py --rows 32,64 --no-prefill-bench --dtype fp8 --json gpurun_out/rows_nb${nb}.jsonl > gpurun_out/rows_nb${nb}.log 2>&1
  VWA_GEMM_NB=$nb timeout -k 10 300 python -u tools/rows_sweep.py --rows 32,64 --no-prefill-bench --json gpurun_out/rows_nb${nb}.jsonl >> gpurun_out/rows_nb${nb}.log 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r_fp8 -o run -- python3 -u tools/rows_sweep.py --rows 32 --iters 10 --no-prefill-bench --dtype fp8 > gpurun_out/r_fp8.log 2>&1
python tools/summarize_profile.py /tmp/r_fp8/run_results.db "rows 32 fp8 (4-stage few-row GEMM)" > gpurun_out/r_fp8.md
