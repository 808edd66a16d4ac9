#!/bin/bash
# Interleaved A/B of engine builds on the headline bench (HBM-resident configs[1]):
# tools/ab_bench.sh <reps> <name=lib-or-env-or-flags>...   e.g. base= v1=build/ab/v1.so full=FDGPU_HALF=0 k4=--overlap,4
# Each run prints one line: name value dsm prep.  Reps alternate the order (ABBA).
reps="$1"; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
for r in $(seq "$reps"); do
  # odd reps run the list forward, even reps backward (ABBA): an order effect cancels over pairs
  if (( r % 2 )); then order=("$@"); else order=(); for (( i=$#; i>=1; i-- )); do order+=("${!i}"); done; fi
  for spec in "${order[@]}"; do
    name="${spec%%=*}"; val="${spec#*=}"
    extra=""
    if [[ "$val" == *.so ]]; then envs="FDGPU_LIB=$val"; elif [[ "$val" == --* ]]; then envs="X=1"; extra="${val//,/ }"; else envs="$val"; fi
    out=$(env $envs timeout -k 10 120 $B $extra 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernel_ms']; print(sys.argv[1], round(d['value']/1e6,2), round(k['dsm'],3), round(k['prep'],3), d['results_ok'])" "$name" "$out" || echo "$name failed"
  done
done
