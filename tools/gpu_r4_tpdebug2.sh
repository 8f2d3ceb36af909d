TPR="python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1"
PT="python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh \
  r4_shape_tests 400 "$PT tests/test_kernels_gpu.py -k tp8_per_rank tests/test_engine_gpu.py::test_chained_layer_tail_matches_per_kernel_path" \
  r4_tp8_70b_nochain2 400 "VWA_CHAIN_TP=0 VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=8 --master-port=29582 tools/tp_check.py" \
  r4_tp4_70b 400 "VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=4 --master-port=29584 tools/tp_check.py"
