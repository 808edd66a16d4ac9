#!/bin/bash
# Max-rate and unreliable legs at 2 vs 3 tiles per GPU, with the tile-loop section profile, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
nproc > gpurun_out/nproc.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/nproc.txt 2>/dev/null; lscpu | head -30 >> gpurun_out/nproc.txt
AB_BASE="--stream-procs 1 --stream-seconds 3 --stream-paced-seconds 1 --stream-unrel-seconds 2 --stream-rates 2e6 --stream-prof" \
  bash tools/gpu_stream_ab.sh tiles3 "--stream-tiles 2" "--stream-tiles 3" "--stream-tiles 2" "--stream-tiles 3"
