set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/x16 -o run -- python3 -u tools/rows_sweep.py --rows 16 --iters 10 --no-prefill-bench > gpurun_out/x16.log 2>&1
python tools/summarize_profile.py /tmp/x16/run_results.db "rows 16 bf16 decode step" > gpurun_out/x16.md
