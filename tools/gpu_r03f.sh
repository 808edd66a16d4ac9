#!/bin/bash
# round 3: tile host-path trims -- the tile GPU tests, then the stream legs (plain and profiled)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_job.sh \
  "tests_tile:600:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_stream_parity.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread"
AB_BASE="--stream-procs 1 --stream-seconds 4 --stream-paced-seconds 2 --stream-unrel-seconds 2 --stream-rates 5e6" \
bash tools/gpu_stream_ab.sh trim "" "--stream-prof"
