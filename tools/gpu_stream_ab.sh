#!/bin/bash
# Stream legs A/B on one box: the bench's stream child (no headline) under a few settings.
# usage: gpurun -- 'bash tools/gpu_stream_ab.sh <tag> "<extra bench args A>" "<extra bench args B>" ...'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag="$1"; shift
mkdir -p gpurun_out/ab_$tag
S="${AB_BASE:---stream-procs 1 --stream-seconds 4 --stream-paced-seconds 3 --stream-unrel-seconds 2 --stream-rates 2e6,10e6}"
i=0; specs=()
for e in "$@"; do
  specs+=("s$i:240:python bench.py --stream-child --stream-token ab$i $S $e > gpurun_out/ab_$tag/s$i.json")
  i=$((i+1))
done
bash tools/gpu_job.sh "${specs[@]}"
