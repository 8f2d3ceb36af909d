# tiled GEMM: numerics (GEMM tests) then the shape table vs hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gemm or linear or swiglu" > gpurun_out/gemm_pytest.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/bench_gemm.py --json gpurun_out/gemm_bench.jsonl > gpurun_out/gemm_bench.log 2>&1 || exit 12
