#!/bin/bash
# A/B of field-arithmetic instruction choices (fd_gpu_f25519.h FD_ADD2 / FD_MAD1 / FD_SQR2_PRE) on the
# HBM-resident configs[1] bench: sigs/s and per-kernel ms for each build/ab/<variant>.so, interleaved
# twice to expose drift.  Build first (CPU): tools/ab_build.sh <variant> -DFD_...=0 ...
# usage (GPU box): bash tools/dsm_ab.sh <variant> ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dsm_ab
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
specs=()
for rep in 1 2; do
  for v in "$@"; do
    specs+=("${v}_$rep:120:FDGPU_LIB=build/ab/$v.so $B > gpurun_out/dsm_ab/${v}_$rep.json")
  done
done
bash tools/gpu_job.sh "${specs[@]}"
