set -e
for r in 1 4; do
  timeout -k 10 120 python tools/chain_probe.py --rows $r --json gpurun_out/probe4.jsonl
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_tiled.log 2>&1
