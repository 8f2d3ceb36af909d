set -e
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_osub.log 2>&1
for x in 1 0; do for r in 1 4; do
  VWA_CHAIN_OSUB=$x timeout -k 10 120 python tools/chain_probe.py --rows $r --attn --json gpurun_out/probe11_o$x.jsonl
done; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_osub.log 2>&1
VWA_CHAIN_OSUB=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_osub0.log 2>&1
