TPR="python -u -m torch.distributed.run --nnodes=1 --master-addr=127.0.0.1"
PT="python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh \
  r4_chain_fix_tests 600 "$PT tests/test_engine_gpu.py -k 'chained or 70b' tests/test_kernels_gpu.py -k 'many_rows or fp8'" \
  r4_tp8_70b_v3 400 "VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 $TPR --nproc-per-node=8 --master-port=29582 tools/tp_check.py" \
  r4_prof_rows32_gemm 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_rows32_gemm -o run -- python3 -u tools/rows_sweep.py --rows 32 --iters 10 --no-prefill-bench" \
  r4_prof_rows8 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_rows8 -o run -- python3 -u tools/rows_sweep.py --rows 8 --iters 10 --no-prefill-bench"
