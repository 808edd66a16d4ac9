#!/bin/bash
# Round-6 GPU jobs: tools/r06_jobs.sh <job>   (each step under its own time limit via tools/gpu_job.sh)
#   first : the restored tree: default bench (line + detail) and the stream / tile parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
job="$1"; shift
T="python -u -m pytest -q -rA --timeout 300 --timeout-method thread"

case "$job" in
  first)
    d=gpurun_out/r06_first; mkdir -p $d
    bash tools/gpu_job.sh \
      "bench:400:python bench.py --detail-out $d/bench_detail.json > $d/bench_line.json" \
      "tests:600:$T tests/test_gpu_stream_parity.py tests/test_gpu_vtile.py tests/test_gpu_stem.py"
    ;;
  *) echo "unknown job $job"; exit 2 ;;
esac
