#!/bin/bash
# A/B of the phase-2 LDS item and xdma pre2 (chain_probe per-layer time), after the chain tests
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "chain" > gpurun_out/t_chain.log 2>&1 || exit $?
for rows in 1 4; do
  for rep in 1 2; do
    for cfg in "0 0" "1 0" "0 1" "1 1"; do
      set -- $cfg
      VWA_CHAIN_LDS_ITEM2=$1 VWA_CHAIN_XPRE2=$2 timeout -k 10 120 python tools/chain_probe.py --rows $rows --attn \
        --json gpurun_out/ab_lds2.jsonl > gpurun_out/ab_last.log 2>&1 || exit $?
      python -c "import json,sys; d=json.loads(open(\"gpurun_out/ab_last.log\").read().strip().splitlines()[-1]); print(\"rows=$rows lds2=$1 xpre2=$2\", d[\"chained_us\"], d[\"stamps_med_us\"])"
    done
  done
done
