#!/bin/bash
# A/B of the SHA-512 message loads (FD_SHA_LOAD 0 = non-temporal, 1 = plain): kernel times and
# FETCH_SIZE of fd_hash_kernel on the HBM-resident configs[1] bench, one rocprofv3 pass per counter.
# usage (GPU box): bash tools/sha_ab.sh   (needs build/ab/shaplain.so: tools/ab_build.sh shaplain -DFD_SHA_LOAD=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-batch 0 --stream-frags 0 --no-extra-configs"
P="timeout -s KILL 120 rocprofv3 --kernel-include-regex fd_ -f csv"
specs=()
for v in nt plain; do
  lib=""; [ "$v" = plain ] && lib="FDGPU_LIB=build/ab/shaplain.so"
  specs+=("stats_$v:180:mkdir -p gpurun_out/sha_$v && $lib rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sha_$v/stats -o run -- $B > gpurun_out/sha_$v/bench.json 2>gpurun_out/sha_$v/bench.err")
  specs+=("fetch_$v:150:$lib $P --pmc FETCH_SIZE -d gpurun_out/sha_$v/fetch -o run -- $B")
done
bash tools/gpu_job.sh "${specs[@]}"
