#!/bin/bash
# Round 4 paced-leg A/B with exclusive latency-path workgroups (the new default): 1 vs 2 paced tiles.  One tile's
# host loop saturates near 10M frags/s (~100 ns per frag); two tiles halve that load, and exclusivity keeps
# their four contexts' batches off each other's SIMDs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04u
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 7.5e6,10e6,12.5e6,15e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04u/$1.json > gpurun_out/r04u/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run t1a '')" "$(run t2a '--stream-lat-tiles 2')" "$(run t2c1a '--stream-lat-tiles 2 --stream-lat-ctx 1')" \
  "$(run t2c1b '--stream-lat-tiles 2 --stream-lat-ctx 1')" "$(run t2b '--stream-lat-tiles 2')" "$(run t1b '')"
