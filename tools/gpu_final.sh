#!/bin/bash
# Round-end evidence on one GPU: the GPU test suite, the default bench, rocprof kernel stats of the
# headline (HBM-resident) bench, and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters).
# usage: gpurun --timeout 1500 -- 'bash tools/gpu_final.sh <tag>'
tag="${1:-final}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
P="timeout -s KILL 120 rocprofv3 --kernel-include-regex fd_ -f csv"
d="gpurun_out/prof_${tag}"
bash "$(dirname "$0")/gpu_job.sh" \
  "tests:1100:python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread" \
  "smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:480:mkdir -p $d && python bench.py --steps 20 --warmup 5 --detail-out $d/bench_detail.json > gpurun_out/bench_${tag}.json" \
  "stats:180:rocprofv3 --kernel-trace --stats -f csv -d $d/stats -o run -- $B > $d/bench_under_rocprof.json" \
  "pmc_fetch:150:$P --pmc FETCH_SIZE -d $d/fetch -o run -- $B" \
  "pmc_write:150:$P --pmc WRITE_SIZE -d $d/write -o run -- $B" \
  "pmc_sq:150:$P --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $d/sq -o run -- $B"
