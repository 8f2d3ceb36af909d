#!/bin/bash
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
VWA_CHAIN_ROT=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "chain" > gpurun_out/t_rot.log 2>&1 || { tail -30 gpurun_out/t_rot.log; exit 1; }
tail -1 gpurun_out/t_rot.log
for rep in 1 2; do
  for f in 0 1; do
    VWA_CHAIN_ROT=$f timeout -k 10 120 python tools/chain_probe.py --rows 1 --attn --json gpurun_out/ab_rot.jsonl > gpurun_out/ab_last.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/ab_last.log').read().strip().splitlines()[-1]); print('rot=$f', d['chained_us'], d['stamps_med_us'], 'gu_end max attn/other', d['attn_wg']['max'][4], d['other_wg']['max'][4])"
  done
done
tools/_ab_env.sh "VWA_CHAIN_ROT=0" "VWA_CHAIN_ROT=1"
