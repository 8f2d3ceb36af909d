#!/bin/bash
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "chain" > gpurun_out/t_xg.log 2>&1 || { tail -40 gpurun_out/t_xg.log; exit 1; }
tail -1 gpurun_out/t_xg.log
tools/_ab_env.sh "VWA_CHAIN_MAX_ROWS=4" "VWA_CHAIN_MAX_ROWS=16"
timeout -k 10 300 env VWA_CHAIN_MAX_ROWS=4 python bench.py --steps 3 --warmup 1 --concurrent 8 > gpurun_out/c8_r4.log 2>&1 || exit $?
timeout -k 10 300 env VWA_CHAIN_MAX_ROWS=16 python bench.py --steps 3 --warmup 1 --concurrent 8 > gpurun_out/c8_r16.log 2>&1 || exit $?
for f in c8_r4 c8_r16; do python -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['concurrent'])"; done
