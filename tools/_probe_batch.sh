set -e
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_early.log 2>&1
for r in 1 4; do
  timeout -k 10 120 python tools/chain_probe.py --rows $r --attn --json gpurun_out/probe9.jsonl
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_early.log 2>&1
