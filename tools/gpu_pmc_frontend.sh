# rocprofv3 hardware-counter passes over tools/pmc_frontend.py (one counter group per run)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 5 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/fe_pmc/p1 -- python -u tools/pmc_frontend.py > gpurun_out/fe_pmc_p1.log 2>&1 || exit 21
timeout -k 5 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/fe_pmc/p2 -- python -u tools/pmc_frontend.py > gpurun_out/fe_pmc_p2.log 2>&1 || exit 22
timeout -k 5 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d gpurun_out/fe_pmc/p3 -- python -u tools/pmc_frontend.py > gpurun_out/fe_pmc_p3.log 2>&1 || exit 23
timeout -k 5 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/fe_pmc/p4 -- python -u tools/pmc_frontend.py > gpurun_out/fe_pmc_p4.log 2>&1 || exit 24
