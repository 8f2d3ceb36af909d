#!/bin/bash
# Run GPU steps in order; stop at the first step that crashed/timed out (exit >= 124 or signal).
# usage: tools/gpu_step.sh "<name>:<timeout>:<cmd>" ...
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout $to) : $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after crash/timeout"; exit $rc; fi
done
exit 0
