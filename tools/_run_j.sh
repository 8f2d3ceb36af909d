PMC1="--pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY"
PMC2="--pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
PMC3="--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
KT="--kernel-trace --output-format csv"
P70="tools/pmc_chain.py --model llama3-70b --layers 3"
bash tools/gpu_steps.sh \
  rows_chain16 300 "VWA_CHAIN_MAX_ROWS=16 python -u tools/rows_sweep.py --rows 1,8,16 --no-prefill-bench --json gpurun_out/rows_chain16.jsonl" \
  bench_c8_chain16 500 "VWA_CHAIN_MAX_ROWS=16 python -u bench.py --concurrent 8 --steps 10 --warmup 3" \
  pmc70_p1 150 "rocprofv3 $PMC1 $KT -d gpurun_out/pmc70/p1 -- python3 -u $P70" \
  pmc70_p2 150 "rocprofv3 $PMC2 $KT -d gpurun_out/pmc70/p2 -- python3 -u $P70" \
  pmc70_p3 150 "rocprofv3 $PMC3 $KT -d gpurun_out/pmc70/p3 -- python3 -u $P70" \
  pmcfp8_p3 150 "rocprofv3 $PMC3 $KT -d gpurun_out/pmcfp8/p3 -- python3 -u tools/pmc_fp8_chain.py" \
  pmcfp8_p1 150 "rocprofv3 $PMC1 $KT -d gpurun_out/pmcfp8/p1 -- python3 -u tools/pmc_fp8_chain.py"
