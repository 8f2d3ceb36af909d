timeout -k 10 200 python tools/_dbg_rt.py > gpurun_out/dbg_rt.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rt.log 2>&1
for rt in "--row-table" "" "--row-table" ""; do
  timeout -k 10 120 python tools/chain_probe.py --rows 1 --attn $rt --json gpurun_out/probe14.jsonl
done
exit 0
