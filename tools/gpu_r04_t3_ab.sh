#!/bin/bash
# Round 4 max-rate A/B with the final stream defaults (bigger gathers on the max legs): 2 vs 3 verify tiles, ABBA x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04z
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04z/$1.json > gpurun_out/r04z/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run t2a '')" "$(run t3a '--stream-tiles 3')" "$(run t3b '--stream-tiles 3')" "$(run t2b '')" \
  "$(run t2c '')" "$(run t3c '--stream-tiles 3')" "$(run t4a '--stream-tiles 4 --stream-producers 2')" "$(run t3p2 '--stream-tiles 3 --stream-producers 2')"
