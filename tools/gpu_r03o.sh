#!/bin/bash
# fd_hashh_kernel at 4 waves per SIMD (FD_HASHH_MINW=4, 128 VGPRs) against the default (159 VGPRs, 3 waves).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 700 bash tools/ab_bench.sh 4 base=build/ab/base.so hh4=build/ab/hh4.so > gpurun_out/hh4_ab.log 2>&1 || exit $?
cat gpurun_out/hh4_ab.log
