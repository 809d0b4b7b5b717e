#!/bin/bash
# Run a sequence of GPU steps; continue only after rc 0/1 (pass / test failure).
# Any other code (fault, abort, segfault, timeout) ends the job immediately.
# usage: scripts/gpu_job.sh "<name>:<timeout_s>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (timeout ${tmo}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
