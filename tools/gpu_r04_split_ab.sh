#!/bin/bash
# Round 4 paced-leg A/B (the knee): each engine context of the paced tile on its own half of the CUs the gathers
# leave (--stream-lat-cu-split 1), so the two staggered batches never share SIMDs; round-4 measurements put
# the two-context chain at ~500 us against ~350 us alone (profiles/r04/k).  First the split's GPU tests, then
# the paced leg at the knee rate under a kernel trace with and without the split, then interleaved legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
P="python3 bench.py --steps 1 --warmup 0 --txns 65536 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2"
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04m/$1.json > gpurun_out/r04m/$1.out\""; }
eval bash tools/gpu_job.sh \
  "\"splitt:300:python -u -m pytest tests/test_gpu_vtile.py -k 'cu_split or stream_run_link' -x -q --timeout 200 --timeout-method thread\"" \
  "\"pprof0:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04m/prof0 -o run -- $P --detail-out gpurun_out/r04m/pprof0.json > gpurun_out/r04m/pprof0.out\"" \
  "\"pprof1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04m/prof1 -o run -- $P --stream-lat-cu-split 1 --detail-out gpurun_out/r04m/pprof1.json > gpurun_out/r04m/pprof1.out\"" \
  "$(run s0a '')" "$(run s1a '--stream-lat-cu-split 1')" "$(run s1b '--stream-lat-cu-split 1')" "$(run s0b '')"
