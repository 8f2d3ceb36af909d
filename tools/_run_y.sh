set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
VWA_SKINNY_XG_ROWS=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "skinny or stream or linear or qkv or swiglu" > gpurun_out/kxg.log 2>&1
for xg in 99 12 8; do
  VWA_SKINNY_XG_ROWS=$xg timeout -k 10 300 python -u tools/rows_sweep.py --rows 8,12,16 --no-prefill-bench --json gpurun_out/rows_xg_$xg.jsonl > gpurun_out/rows_xg_$xg.log 2>&1
done
