#!/bin/bash
# Round 4 max-rate A/B: gather size of the max-rate legs (--stream-tput-copy-wait-us / --stream-tput-max-uncopied;
# default now 200 us / 64K).  tools/gatherprobe (profiles/r02/stream/gather_probe.log): with the write-back a
# gather moves 30 GB/s at 4K records, 36 at 16K, 41 at 64K; the stream's two tiles reach ~30 GB/s together.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04s
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04s/$1.json > gpurun_out/r04s/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run old1 '--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0')" "$(run d1 '')" \
  "$(run w500a '--stream-tput-copy-wait-us 500 --stream-tput-max-uncopied 131072')" \
  "$(run w1ka '--stream-tput-copy-wait-us 1000 --stream-tput-max-uncopied 131072')" \
  "$(run w1kb '--stream-tput-copy-wait-us 1000 --stream-tput-max-uncopied 131072')" \
  "$(run w500b '--stream-tput-copy-wait-us 500 --stream-tput-max-uncopied 131072')" "$(run d2 '')" \
  "$(run old2 '--stream-tput-copy-wait-us 0 --stream-tput-max-uncopied 0')"
