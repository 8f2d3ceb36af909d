# DP bench path rehearsal on a 1-GPU box: 2 ranks (gloo control plane) sharing GPU 0 under the
# driver's torchrun launch, no persistent chained launch (two persistent grids cannot be
# co-resident on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VWA_DIST_BACKEND=gloo VWA_CHAIN=0 timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 > gpurun_out/dp2_rehearsal.log 2>&1 || exit 11
