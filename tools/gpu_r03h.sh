#!/bin/bash
# Deferred write-back: GPU tests over the tile paths, then stream legs with the gathered records written
# back by the finish kernel (default) against the gather kernel (round 3's earlier path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_job.sh "tests_raw:600:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_stream_parity.py tests/test_gpu_txn.py tests/test_gpu_faults.py tests/test_gpu_callers.py -x -q --timeout 300 --timeout-method thread" || exit $?
AB_BASE="--stream-procs 1 --stream-seconds 3 --stream-paced-seconds 3 --stream-unrel-seconds 2 --stream-rates 2e6,5e6,10e6" \
  bash tools/gpu_stream_ab.sh defer "--stream-writeback finish" "--stream-writeback gather" "--stream-writeback finish" "--stream-writeback gather"
