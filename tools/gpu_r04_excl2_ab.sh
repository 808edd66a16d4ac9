#!/bin/bash
# Round 4 paced-leg A/B of the exclusivity variants (fdgpu_ed25519_set_cu_exclusive): 1 prep and walk alone on their
# CU (knee 10M but a p99 tail at 5M from gathers that start up to 0.5 ms late, profiles/r04/o), 2 at most two per
# CU, 3 the walk only, 4 the prep only; 0 = off.  Interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04p
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 2e6,5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04p/$1.json > gpurun_out/r04p/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run x0a '')" "$(run x1a '--stream-cu-exclusive 1')" "$(run x2a '--stream-cu-exclusive 2')" \
  "$(run x3a '--stream-cu-exclusive 3')" "$(run x4a '--stream-cu-exclusive 4')" \
  "$(run x4b '--stream-cu-exclusive 4')" "$(run x3b '--stream-cu-exclusive 3')" "$(run x2b '--stream-cu-exclusive 2')" \
  "$(run x1b '--stream-cu-exclusive 1')" "$(run x0b '')"
