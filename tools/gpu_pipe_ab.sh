#!/bin/bash
# headline A/B: consecutive 1M-signature steps on one context vs alternating over two (--pipe 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
mkdir -p gpurun_out
for r in 1 2 3; do
  for p in 1 2 3; do
    out=$(timeout -k 10 180 $B --pipe $p 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernel_ms']; print('pipe', sys.argv[1], round(d['value']/1e6,2), round(d['ms_per_step'],3), round(k['dsm'],3), round(k['prep'],3), d['results_ok'])" "$p" "$out" || echo "pipe $p failed"
  done
done
