#!/bin/bash
# Round 4: the new stream defaults (link in transparent huge pages, 4 records per gather workgroup) through the
# vtile / fault / stream-parity GPU tests, then an interleaved A/B of which CUs the gathers are confined to
# (the last 16 = default, every 16th, the first 16) with round 3's gather setup (4 KiB pages, 1 record per
# workgroup) as a reference arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04j
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 7.5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04j/$1.json > gpurun_out/r04j/$1.out\""; }
eval bash tools/gpu_job.sh \
  "\"vt:400:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_faults.py tests/test_gpu_stream_parity.py -x -q --timeout 200 --timeout-method thread\"" \
  "$(run base1 '')" "$(run spr1a '--stream-gather-cu-spread 1')" "$(run first1a '--stream-gather-cu-spread 2')" \
  "$(run r3a '--stream-no-huge --stream-gather-rpb 1')" "$(run r3b '--stream-no-huge --stream-gather-rpb 1')" \
  "$(run first1b '--stream-gather-cu-spread 2')" "$(run spr1b '--stream-gather-cu-spread 1')" "$(run base2 '')"
