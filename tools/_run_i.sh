bash tools/gpu_steps.sh \
  tp8_70b_v4 500 "VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1 --nproc-per-node=8 --master-port=29578 tools/tp_check.py"
bash tools/gpu_recipes.sh bench
