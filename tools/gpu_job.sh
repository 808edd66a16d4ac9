#!/bin/bash
# Run GPU steps in order; each has its own time limit.  Continue past an
# ordinary failure (exit 1: failing test), stop at anything that smells of
# a fault, abort or timeout (124/134/137/139/...).
# usage: tools/gpu_job.sh "<name>:<timeout_s>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] timeout=${to}s: $cmd" | tee -a gpurun_out/job.log
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/job.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
