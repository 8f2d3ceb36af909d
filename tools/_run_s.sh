set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "handoff or one_launch or tiled_mfma or 8phase or fp8 or qkv or gemm or shared_prefix or decode_attention" > gpurun_out/kt.log 2>&1
timeout -k 10 300 python -u tools/rows_sweep.py --no-prefill-bench --dtype fp8 --json gpurun_out/rows_v_fp8.jsonl > gpurun_out/rows_v.log 2>&1
timeout -k 10 300 python -u tools/rows_sweep.py --json gpurun_out/rows_v_bf16.jsonl >> gpurun_out/rows_v.log 2>&1
timeout -k 10 500 python -u bench.py --dtype fp8 --concurrent 32 --steps 10 --warmup 3 > gpurun_out/bench_v_c32.log 2>&1
timeout -k 10 500 python -u bench.py --concurrent 8 --steps 10 --warmup 3 > gpurun_out/bench_v_c8.log 2>&1
