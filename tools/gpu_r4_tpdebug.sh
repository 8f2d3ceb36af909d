# 70B TP=8 debugging + the rows sweep (decode step vs rows, batched admission prefill)
TPR="python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1"
bash tools/gpu_steps.sh \
  r4_rows_sweep 400 "python -u tools/rows_sweep.py --json gpurun_out/r4_rows_sweep.jsonl" \
  r4_70b_griddiv8 300 "VWA_CHAIN_GRID_DIV=8 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu tests/test_engine_gpu.py -k 70b" \
  r4_tp2_70b 400 "VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=2 --master-port=29581 tools/tp_check.py" \
  r4_tp8_70b_nochain 400 "VWA_CHAIN_TP=0 VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=8 --master-port=29582 tools/tp_check.py" \
  r4_tp8_70b_noattn 400 "VWA_CHAIN_ATTN=0 VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=8 --master-port=29583 tools/tp_check.py"
