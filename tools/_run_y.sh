set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 1 0; do
  VWA_PREFILL_FLASH=$f timeout -k 10 300 python -u tools/rows_sweep.py --rows 32 --dtype fp8 --json gpurun_out/rows_z_fp8_$f.jsonl > gpurun_out/rows_z_$f.log 2>&1
  VWA_PREFILL_FLASH=$f timeout -k 10 300 python -u tools/rows_sweep.py --rows 64 --json gpurun_out/rows_z_bf16_$f.jsonl >> gpurun_out/rows_z_$f.log 2>&1
done
timeout -k 10 500 python -u bench.py > gpurun_out/bench_z_bf16.log 2>&1
