#!/bin/bash
# Round-end style GPU session plus a kernel-trace profile of the latency
# path (small batches: fd_prep_kernel, fd_dsm4_kernel / fd_dsm2_kernel).
# usage: gpurun --timeout 1100 -- 'bash tools/gpu_round2.sh <tag>'
tag="${1:-run}"
bash "$(dirname "$0")/gpu_round.sh" "$tag" && \
bash "$(dirname "$0")/gpu_job.sh" \
  "latprof:180:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${tag}/lat -o run -- python3 tools/latency_probe.py 8192 16384 32768"
