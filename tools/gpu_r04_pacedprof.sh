#!/bin/bash
# Round 4: the paced leg's kernel chain under a kernel trace (10M frags/s, one tile, 2 contexts: the knee's
# rate), to compare each kernel's duration in the stream with the isolated chain (profiles/r03/latency_chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "pprof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r04l/prof -o run -- python3 bench.py --steps 1 --warmup 0 --txns 65536 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2 --detail-out gpurun_out/r04l/pprof.json > gpurun_out/r04l/pprof.out"
