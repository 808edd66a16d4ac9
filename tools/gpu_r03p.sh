#!/bin/bash
# The two prep trims together (SHA-512 full-block fast path + one-pass fe_pack) against the build before them,
# ABBA over 6 reps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 bash tools/ab_bench.sh 6 before=build/ab/before.so after=build/ab/after.so > gpurun_out/trims_abba.log 2>&1 || exit $?
cat gpurun_out/trims_abba.log
