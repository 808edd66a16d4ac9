#!/bin/bash
# Round 4 max-rate A/B on the final build: bigger gathers.  The gather streams are ~87 % busy at the max rate
# (profiles/r04/final: 17K gathers/s of ~1,330 records, 101 us each); a gather's fixed cost is amortised over
# more records when copies start later (--stream-copy-wait-us, default 50) with a larger uncopied bound.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04r
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04r/$1.json > gpurun_out/r04r/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run b1 '')" "$(run w100a '--stream-copy-wait-us 100 --stream-max-uncopied 32768')" \
  "$(run w200a '--stream-copy-wait-us 200 --stream-max-uncopied 65536')" "$(run u32a '--stream-max-uncopied 32768')" \
  "$(run u32b '--stream-max-uncopied 32768')" "$(run w200b '--stream-copy-wait-us 200 --stream-max-uncopied 65536')" \
  "$(run w100b '--stream-copy-wait-us 100 --stream-max-uncopied 32768')" "$(run b2 '')"
