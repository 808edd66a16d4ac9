#!/bin/bash
# Round 4 paced-leg A/B (the knee), interleaved on one box: engine contexts per paced tile.  With 2 contexts
# a batch launches while the other context's batch is still running (the two share the chip, each chain runs
# ~500 us instead of ~330 us); with 1 the next batch fills while the current one runs.  Arms: 2 (default),
# 1, 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04k
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04k/$1.json > gpurun_out/r04k/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run c2a '')" "$(run c1a '--stream-lat-ctx 1')" "$(run c3a '--stream-lat-ctx 3')" \
  "$(run c3b '--stream-lat-ctx 3')" "$(run c1b '--stream-lat-ctx 1')" "$(run c2b '')"
