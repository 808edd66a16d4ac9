#!/bin/bash
# Kernel trace only (no API trace: that slowed the stream 50x) of the stream's cal + max legs, reduced on
# the box by tools/trace_queue.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=gpurun_out/ktrace_${1:-1}; shift
mkdir -p $d
bash tools/gpu_job.sh \
  "ktrace:300:rocprofv3 --kernel-trace -f csv -d $d/t -o run -- python bench.py --stream-child --stream-token kt --stream-procs 1 --stream-seconds 2 --stream-rates '' --stream-unrel-seconds 1 $* > $d/legs.json" \
  "reduce:200:python tools/trace_queue.py $d --drop > $d/reduce.log"
