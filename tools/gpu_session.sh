#!/bin/bash
# Runs a list of GPU steps; each step has its own time limit.  Stops the whole
# session after a fault/abort/segfault/timeout (exit 124/134/137/139 or >128),
# continues after ordinary failures (exit 1/2: test failures, Python errors).
# usage: tools/gpu_session.sh "<name>|<timeout_s>|<cmd>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; tmo="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${tmo}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] ; then
    echo "=== stopping session after rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
