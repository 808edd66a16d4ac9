#!/bin/bash
# Profile passes only (kernel-trace stats + separate PMC passes) of the
# HBM-resident bench (no stream leg, no CPU baseline).
# usage: gpurun --timeout 900 -- 'bash tools/gpu_prof.sh <tag>'
tag="${1:-run}"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
P="timeout -s KILL 90 rocprofv3 --kernel-include-regex fd_ -f csv"
bash "$(dirname "$0")/gpu_job.sh" \
  "stats:180:mkdir -p gpurun_out/prof_${tag} && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${tag}/stats -o run -- $B > gpurun_out/prof_${tag}/bench_under_rocprof.log 2>&1" \
  "pmc_fetch:120:$P --pmc FETCH_SIZE -d gpurun_out/prof_${tag}/fetch -o run -- $B" \
  "pmc_write:120:$P --pmc WRITE_SIZE -d gpurun_out/prof_${tag}/write -o run -- $B" \
  "pmc_sq:120:$P --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/prof_${tag}/sq -o run -- $B"
