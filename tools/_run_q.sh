set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "shared_prefix or row_groups or decode_attention or one_launch or quant_fp8_rows or tiled_mfma or 8phase or fp8 or qkv" > gpurun_out/kt.log 2>&1
timeout -k 10 200 python -u tools/attn_probe.py --impls mq --only-llama > gpurun_out/attn_q.log 2>&1
timeout -k 10 300 python -u tools/rows_sweep.py --rows 8,16,32,64 --no-prefill-bench --dtype fp8 --json gpurun_out/rows_q_fp8.jsonl > gpurun_out/rows_q.log 2>&1
timeout -k 10 300 python -u tools/rows_sweep.py --rows 8,16,32,64 --no-prefill-bench --json gpurun_out/rows_q_bf16.jsonl >> gpurun_out/rows_q.log 2>&1
for dt in fp8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/q_${dt} -o run -- python3 -u tools/rows_sweep.py --rows 32 --iters 10 --no-prefill-bench --dtype $dt > gpurun_out/q_${dt}.log 2>&1
  python tools/summarize_profile.py /tmp/q_${dt}/run_results.db "rows 32 $dt (QKV rope in the reduce, shared-prefix attention)" > gpurun_out/q_${dt}.md
done
