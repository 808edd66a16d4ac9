#!/bin/bash
# One-pass fe_pack: the whole GPU suite, then an interleaved headline A/B against the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_job.sh "tests:1100:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" || exit $?
timeout -k 10 600 bash tools/ab_bench.sh 3 old=build/ab/packold.so new=build/ab/packnew.so > gpurun_out/pack_ab.log 2>&1 || exit $?
cat gpurun_out/pack_ab.log
