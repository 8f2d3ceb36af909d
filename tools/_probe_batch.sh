set -e
for ip in 2 0; do for r in 1 4; do
  VWA_CHAIN_IDLE_PRE=$ip timeout -k 10 120 python tools/chain_probe.py --rows $r --attn --json gpurun_out/probe8_ip$ip.jsonl
done; done
