#!/bin/bash
# Round 4 host-loop A/B: one clock_gettime per tile-loop pass (this build) vs two (the previous build,
# firedancer_amd/ab_vtile_old.so via FDGPU_VTILE_LIB).  At a paced rate a pass often takes a single frag.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04w
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 7.5e6,10e6,12.5e6,15e6 --stream-paced-seconds 2 --stream-seconds 4 --stream-unrel-seconds 1"
run() { echo "\"$1:200:$3 $S $2 --detail-out gpurun_out/r04w/$1.json > gpurun_out/r04w/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run new1 '')" "$(run old1 '' FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so)" \
  "$(run old2 '' FDGPU_VTILE_LIB=firedancer_amd/ab_vtile_old.so)" "$(run new2 '')"
