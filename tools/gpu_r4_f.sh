TPR="python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1"
PT="python -u -m pytest -v --timeout 250 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh \
  r4_new_kernel_tests 400 "$PT tests/test_kernels_gpu.py -k 'fp8 or many_rows or tp8_per_rank or tiled_weights or skinny'" \
  r4_rows_sweep_v2 300 "python -u tools/rows_sweep.py --json gpurun_out/r4_rows_sweep_v2.jsonl" \
  r4_tp8_trace 400 "VWA_TP_CHECK_TRACE=1 VWA_CHAIN_TP=0 VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=8 --master-port=29582 tools/tp_check.py" \
  r4_chain_tp8rank 300 "$PT 'tests/test_engine_gpu.py::test_chained_layer_tail_matches_per_kernel_path[llama70b-tp8-rank-griddiv8]'" \
  r4_prof_rows32 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_rows32 -o run -- python3 -u tools/rows_sweep.py --rows 32 --iters 6"
