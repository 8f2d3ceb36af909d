set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "2 0 100" "2 0 75" "2 0 50" "4 0 50"; do
  set -- $cfg
  VWA_GEMM_NB=$1 VWA_ROWQ_HANDOFF=$2 VWA_GEMM_SPLIT_FILL=$3 timeout -k 10 200 python -u tools/rows_sweep.py --rows 32,64 --no-prefill-bench --dtype fp8 --json gpurun_out/ab_u_${1}_${2}_${3}.jsonl > gpurun_out/ab_u_${1}_${2}_${3}.log 2>&1
done
for cfg in "2 100" "2 75" "4 75" "4 50" "2 50"; do
  set -- $cfg
  VWA_GEMM_NB=$1 VWA_GEMM_SPLIT_FILL=$2 timeout -k 10 200 python -u tools/rows_sweep.py --rows 32,64 --no-prefill-bench --json gpurun_out/ab_u_bf16_${1}_${2}.jsonl > gpurun_out/ab_u_bf16_${1}_${2}.log 2>&1
done
