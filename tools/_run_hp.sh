set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py > gpurun_out/ke.log 2>&1
timeout -k 10 500 python -u bench.py --dtype fp8 --concurrent 32 --steps 10 --warmup 3 > gpurun_out/bench_h_c32.log 2>&1
timeout -k 10 500 python -u bench.py --concurrent 8 --steps 10 --warmup 3 > gpurun_out/bench_h_c8.log 2>&1
