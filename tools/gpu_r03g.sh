#!/bin/bash
# round 3: finish kernel with one wave per image -- raw-path tests, one-batch probe, stream legs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_job.sh \
  "tests_raw:600:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_stream_parity.py tests/test_gpu_txn.py tests/test_gpu_faults.py tests/test_gpu_callers.py -x -q --timeout 300 --timeout-method thread" \
  "raw:200:python tools/raw_batch_probe.py 512 1536 4096 > gpurun_out/rawprobe_g.jsonl"
cat gpurun_out/rawprobe_g.jsonl
AB_BASE="--stream-procs 1 --stream-seconds 3 --stream-paced-seconds 3 --stream-unrel-seconds 2 --stream-rates 2e6,5e6,10e6" \
bash tools/gpu_stream_ab.sh fin "" ""
