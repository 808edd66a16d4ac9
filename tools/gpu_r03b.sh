#!/bin/bash
# round 3, second GPU call: sandbox probe, stream write-back A/B, VALU issue probe, decode fold A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/stream_parity.log 2>&1; tail -5 gpurun_out/stream_parity.log
bash tools/gpu_sandbox.sh
bash tools/gpu_stream_ab.sh wb "--stream-gather-cus 16" "--stream-gather-cus 16 --stream-writeback none" "--stream-gather-cus 0 --stream-writeback none" "--stream-gather-cus 32 --stream-writeback none"
bash tools/gpu_instprobe.sh
timeout -k 10 400 bash tools/ab_bench.sh 3 base=build/ab/base.so dec0=build/ab/dec0.so > gpurun_out/ab_dec0.log 2>&1
cat gpurun_out/ab_dec0.log
