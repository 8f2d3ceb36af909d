# 32 concurrent sessions (bf16): kernel trace of the continuous-batching steady state
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/conc_prof -o run -- python -u bench.py --concurrent 32 --steps 2 --warmup 1 > gpurun_out/conc_prof.log 2>&1 || exit 11
