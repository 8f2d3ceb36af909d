# round-3 GPU benchmark pass: headline, fp8 + 32 sessions (config 5), bf16 + 8 sessions, rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench_bf16.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py --dtype fp8 --concurrent 32 --steps 10 --warmup 3 > gpurun_out/r3_bench_fp8_c32.log 2>&1 || exit 12
timeout -k 10 400 python -u bench.py --concurrent 8 --steps 10 --warmup 3 > gpurun_out/r3_bench_bf16_c8.log 2>&1 || exit 13
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_prof_bf16 -o run -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/r3_prof_bf16.log 2>&1 || exit 14
