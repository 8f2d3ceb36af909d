# Two-rank tensor-parallel check (tools/tp_check.py) on ONE GPU, each rank under its own
# rocprofv3 --kernel-trace (no launcher in between: the ranks are plain children of this shell),
# so the per-rank kernel traces show the chained decode layer's launches at TP=2.
#   bash tools/gpu_tp_prof.sh   (on the GPU box; outputs under gpurun_out/r3_tp_prof/)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_tp_prof/rank$r -o run \
    -- python3 tools/tp_check.py > gpurun_out/r3_tp_prof_rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc
