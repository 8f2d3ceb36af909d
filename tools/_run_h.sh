PT="python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu"
bash tools/gpu_steps.sh \
  r4_chain_fix_tests 700 "$PT tests/test_engine_gpu.py -k 'chained or 70b' tests/test_kernels_gpu.py -k 'many_rows or fp8 or tp8'" \
  r4_prof_rows32_gemm 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_rows32_gemm -o run -- python3 -u tools/rows_sweep.py --rows 32 --iters 10 --no-prefill-bench" \
  r4_prof_rows8 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_rows8 -o run -- python3 -u tools/rows_sweep.py --rows 8 --iters 10 --no-prefill-bench"
bash tools/gpu_recipes.sh tp
