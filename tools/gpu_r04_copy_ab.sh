#!/bin/bash
# Round 4 max-rate A/B: host-copy intake (--stream-copy: the tile copies each record into its out dcache as the
# reference's during_frag does, and each batch goes up in one DMA of its contiguous out-dcache range) against
# zero-copy intake (GPU gathers + writes back: ~30 GB/s each way of PCIe, profiles/r04/x), at 2 / 3 / 4 tiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04y
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6 --stream-paced-seconds 1 --stream-seconds 4 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04y/$1.json > gpurun_out/r04y/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run zc2 '')" "$(run cp2 '--stream-copy')" "$(run cp3 '--stream-copy --stream-tiles 3')" \
  "$(run cp4 '--stream-copy --stream-tiles 4')" "$(run zc3 '--stream-tiles 3')"
