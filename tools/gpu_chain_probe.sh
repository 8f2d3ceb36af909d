# chained decode layer: per-phase stamps bf16 / fp8, with and without barrier waits (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "" "--fp8"; do
  timeout -k 10 120 python -u tools/chain_probe.py --attn $v > gpurun_out/cp_attn${v// /}.log 2>&1 || exit 11
  timeout -k 10 120 python -u tools/chain_probe.py --attn --no-wait $v > gpurun_out/cp_attn_nowait${v// /}.log 2>&1 || exit 12
done
