#!/bin/bash
# Prep-kernel occupancy A/B (headline, interleaved) and the tile loop's prefetch distance (stream legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_bench.sh 2 base= sha4=build/ab/sha4.so sha3=build/ab/sha3.so dec5=build/ab/dec5.so \
  hh4=build/ab/hh4.so > gpurun_out/prep_ab.log 2>&1 || exit $?
cat gpurun_out/prep_ab.log
AB_BASE="--stream-procs 1 --stream-seconds 3 --stream-paced-seconds 3 --stream-unrel-seconds 2 --stream-rates 2e6,10e6" \
  bash tools/gpu_stream_ab.sh pf "--stream-pf-dist 1" "--stream-pf-dist 4" "--stream-pf-dist 8" "--stream-pf-dist 1" "--stream-pf-dist 4" "--stream-pf-dist 8"
