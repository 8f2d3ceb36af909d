# rocprofv3 hardware-counter passes over tools/pmc_kernels.py (one counter group per run; pass
# limits: <= 8 SQ, 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), 2 GRBM per pass) + a kernel-trace
# profile of the headline bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 5 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/r3_pmc/p1 -- python -u tools/pmc_kernels.py > gpurun_out/r3_pmc_p1.log 2>&1 || exit 21
timeout -k 5 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/r3_pmc/p2 -- python -u tools/pmc_kernels.py > gpurun_out/r3_pmc_p2.log 2>&1 || exit 22
timeout -k 5 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r3_pmc/p3 -- python -u tools/pmc_kernels.py > gpurun_out/r3_pmc_p3.log 2>&1 || exit 23
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_bf16 -o run -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3_prof_bf16.log 2>&1 || exit 24
