# rocprofv3 counter passes over the fp8 chained decode layer (tools/pmc_fp8_chain.py)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 5 120 python -u tools/pmc_fp8_chain.py > gpurun_out/fp8pmc_plain.log 2>&1 || exit 20
timeout -k 5 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/fp8_pmc/p1 -- python -u tools/pmc_fp8_chain.py > gpurun_out/fp8pmc_p1.log 2>&1 || exit 21
timeout -k 5 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/fp8_pmc/p2 -- python -u tools/pmc_fp8_chain.py > gpurun_out/fp8pmc_p2.log 2>&1 || exit 22
timeout -k 5 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d gpurun_out/fp8_pmc/p3 -- python -u tools/pmc_fp8_chain.py > gpurun_out/fp8pmc_p3.log 2>&1 || exit 23
