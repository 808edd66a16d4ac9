#!/bin/bash
# SHA-512 Ch as v_bitop3_b32: the whole GPU suite, then an ABBA headline A/B against the v_bfi_b32 build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_job.sh "tests:1100:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" || exit $?
timeout -k 10 700 bash tools/ab_bench.sh 4 old=build/ab/chold.so new=build/ab/chnew.so > gpurun_out/ch_ab.log 2>&1 || exit $?
cat gpurun_out/ch_ab.log
