# A/B: headline bench with the 8-phase prompt GEMM (default routing) vs the 128x128 kernel only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VWA_GEMM_P8=0 timeout -k 10 300 python -u bench.py > gpurun_out/ab_p8_off.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > gpurun_out/ab_p8_on.log 2>&1 || exit 12
