#!/bin/bash
# Round 4: repeat of the exclusivity A/B (off vs prep and walk alone on their CUs) on another box, at the default
# paced rates (2 / 5 / 7.5 / 10 / 15M frags/s), three interleaved pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04q
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04q/$1.json > gpurun_out/r04q/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run y0a '')" "$(run y1a '--stream-cu-exclusive 1')" "$(run y1b '--stream-cu-exclusive 1')" "$(run y0b '')" \
  "$(run y0c '')" "$(run y1c '--stream-cu-exclusive 1')"
