#!/bin/bash
# Same-box bench A/B of environment settings: tools/_ab_env.sh "<ENV=.. ENV=..>" "<ENV=..>" ... (two rounds)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/ab_env_last.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/ab_env_last.log').read().strip().splitlines()[-1]); print('$cfg |', d['value'], d['llm_decode_steps_mean'], d['decode_iteration_host_us']['gpu_wait_us'])" | tee -a gpurun_out/ab_env.txt
  done
done
