# front-end kernels: numerics (kernel + engine GPU tests), microbenchmark vs torch library ops
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fe_pytest.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/bench_frontend.py --json gpurun_out/frontend.jsonl > gpurun_out/fe_bench.log 2>&1 || exit 12
