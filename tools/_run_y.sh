set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --concurrent 8 --steps 10 --warmup 3 > gpurun_out/bench_b_c8.log 2>&1
