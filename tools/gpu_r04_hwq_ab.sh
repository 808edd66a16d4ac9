#!/bin/bash
# Round 4 stream A/B, interleaved (ABC..CBA) on one box: the tile processes' hardware queues.  HIP spreads a
# process's streams over GPU_MAX_HW_QUEUES (default 4) hardware queues; a tile context has a compute and a
# gather stream, so 2 tiles x 2 contexts (paced) or 3 tiles (max rate) put streams on shared queues, where a
# packet waits behind another stream's.  Arms: the default; 8 queues; 2 paced tiles on 4 / on 8 queues;
# 3 max-rate tiles on 12 queues; the tiles pinned to the lowest cores of the GPU's node without the idle-core
# sample (FDGPU_LINK_PIN=lowest, round 3's placement).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04h
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$3 $S $2 --detail-out gpurun_out/r04h/$1.json > gpurun_out/r04h/$1.out\""; }
eval bash tools/gpu_job.sh \
  "\"vt:400:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_faults.py tests/test_gpu_stream_parity.py -x -q --timeout 200 --timeout-method thread\"" \
  "$(run base1 '')" "$(run q8a '--stream-hw-queues 8')" "$(run lt2a '--stream-lat-tiles 2')" \
  "$(run lt2q8a '--stream-lat-tiles 2 --stream-hw-queues 8')" "$(run t3q12a '--stream-tiles 3 --stream-hw-queues 12')" \
  "$(run low1 '' FDGPU_LINK_PIN=lowest)" "$(run low2 '' FDGPU_LINK_PIN=lowest)" "$(run t3q12b '--stream-tiles 3 --stream-hw-queues 12')" "$(run lt2q8b '--stream-lat-tiles 2 --stream-hw-queues 8')" \
  "$(run lt2b '--stream-lat-tiles 2')" "$(run q8b '--stream-hw-queues 8')" "$(run base2 '')"
