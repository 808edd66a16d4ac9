#!/bin/bash
# cgroup CPU throttling during the stream legs: cpu.stat before and after one stream child, plus the
# threads of the stream process sampled mid-run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cpustat
cat /sys/fs/cgroup/cpu.stat > gpurun_out/cpustat/before.txt
timeout -k 10 240 python bench.py --stream-child --stream-token cs --stream-procs 1 --stream-seconds 3 --stream-paced-seconds 3 \
  --stream-unrel-seconds 2 --stream-rates 2e6,7.5e6,10e6 > gpurun_out/cpustat/legs.json &
pid=$!
for i in 1 2 3 4 5 6 7 8; do
  sleep 3
  cat /sys/fs/cgroup/cpu.stat > gpurun_out/cpustat/mid_$i.txt
  ps -L -o pid,tid,psr,pcpu,stat,comm -p $pid > gpurun_out/cpustat/threads_$i.txt 2>/dev/null
done
wait $pid; rc=$?
cat /sys/fs/cgroup/cpu.stat > gpurun_out/cpustat/after.txt
exit $rc
