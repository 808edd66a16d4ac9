#!/bin/bash
# Call gpurun; if (and only if) the call never reached a GPU box -- gpurun
# reports status=transient (infrastructure side, nothing ran, nothing
# charged) -- wait the advised back-off and call again, at most 6 times.
# Never retries a command that actually ran (pass or fail).
for attempt in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | tail -40
  if echo "$out" | grep -q "status=transient"; then
    wait_s=$(echo "$out" | grep -oE "retry in [0-9]+s" | grep -oE "[0-9]+" | head -1)
    wait_s=${wait_s:-60}
    echo "[gpurun_retry] transient (attempt $attempt), sleeping $((wait_s+10))s"
    sleep $((wait_s+10))
    continue
  fi
  exit $rc
done
exit 3
