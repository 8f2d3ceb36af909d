set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/svc_dbg.jsonl
timeout -k 10 600 python -u tools/service_bench.py --sessions 1 --debounce 0 --chain 1,0,1,0 --json gpurun_out/svc_dbg.jsonl > gpurun_out/svc_dbg.log 2>&1
