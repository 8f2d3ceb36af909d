# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# A step that fails NORMALLY (exit 1: a Python exception / failed check) does not stop the run;
# a fault, abort, segfault or time limit (any other non-zero status) ends it at once.
#   usage: bash tools/gpu_steps.sh name1 secs1 'cmd1' [name2 secs2 'cmd2' ...]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
worst=0
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "[steps] $name: $cmd" >&2
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[steps] $name rc=$rc" >&2
  echo "$name rc=$rc" >> gpurun_out/steps_status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && worst=1
done
exit $worst
