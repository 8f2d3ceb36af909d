#!/bin/bash
# Same-box bench A/B of chain knobs: "LDS_ITEM2 AFLAG" pairs, alternating, two rounds
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "chain" > gpurun_out/t_chain2.log 2>&1 || { tail -30 gpurun_out/t_chain2.log; exit 1; }
tail -1 gpurun_out/t_chain2.log
for rep in 1 2; do
  for cfg in "0 0" "1 0" "1 1"; do
    set -- $cfg
    VWA_CHAIN_LDS_ITEM2=$1 VWA_CHAIN_AFLAG=$2 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/ab_bench_last.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/ab_bench_last.log').read().strip().splitlines()[-1]); print('lds2=$1 aflag=$2', d['value'], d['llm_decode_steps_mean'], d['decode_iteration_host_us']['gpu_wait_us'])" | tee -a gpurun_out/ab_bench.txt
  done
done
