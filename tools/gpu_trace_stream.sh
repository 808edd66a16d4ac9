#!/bin/bash
# Kernel + HIP API trace of short stream legs, reduced on the box to the launch -> start delays
# (tools/trace_gather.py; the raw CSVs are too large to bring back).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=gpurun_out/trace_${1:-1}; shift
mkdir -p $d
bash tools/gpu_job.sh \
  "trace:300:rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $d/t -o run -- python bench.py --stream-child --stream-token tr --stream-procs 1 --stream-frags 3000000 --stream-rates 1e7 $* > $d/legs.json" \
  "reduce:120:python tools/trace_gather.py $d --drop > $d/reduce.log"
