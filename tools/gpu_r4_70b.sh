# round 4, config 4 on one MI355X: 70B-shape chained-layer GPU test, Llama-3-70B bf16 at TP=1
# through bench.py (141 GB of weights in 288 GB of HBM), an 8-rank TP=8 tp_check with 70B per-rank
# shapes sharing the GPU, a kernel trace and HBM counters of the 70B chained layer.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_engine_gpu.py -k "70b or chained_layer_tail" > gpurun_out/r4_70b_pytest.log 2>&1 || exit 11
timeout -k 10 500 python -u bench.py --llm llama3-70b --steps 5 --warmup 2 --verbose > gpurun_out/r4_bench_70b.log 2>&1 || exit 12
VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29571 tools/tp_check.py > gpurun_out/r4_tp8_70b.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof_chain70 -o run -- python3 -u tools/pmc_chain.py --model llama3-70b --layers 3 > gpurun_out/r4_prof_chain70.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/r4_pmc70/p1 -- python3 -u tools/pmc_chain.py --model llama3-70b --layers 3 > gpurun_out/r4_pmc70_p1.log 2>&1 || exit 15
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/r4_pmc70/p2 -- python3 -u tools/pmc_chain.py --model llama3-70b --layers 3 > gpurun_out/r4_pmc70_p2.log 2>&1 || exit 16
