# Whisper-tiny chained decoder with smaller persistent grids (VWA_CHAIN_GRID_DIV)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in 1 4 8 16; do
  VWA_CHAIN_GRID_DIV=$d timeout -k 10 200 python -u tools/asr_timing.py --asr whisper-tiny --reps 5 > gpurun_out/asr_grid_$d.log 2>&1 || exit 11
done
