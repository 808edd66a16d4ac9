#!/bin/bash
# Round 4: kernel traces of the paced leg's tile process itself (bench.py --stream-child under rocprofv3), at the
# knee's 10M frags/s: 2 contexts on all CUs (default), 2 contexts on disjoint CU halves, 1 context.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
C="python3 bench.py --stream-child --stream-device 0 --stream-proc 0 --stream-procs 1 --stream-token pp --stream-seed 1234 --txns 65536 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2"
bash tools/gpu_job.sh \
  "cp0:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c2 -o run -- $C > gpurun_out/r04n/c2.out" \
  "cp1:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c2split -o run -- $C --stream-lat-cu-split 1 > gpurun_out/r04n/c2split.out" \
  "cp2:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c1 -o run -- $C --stream-lat-ctx 1 > gpurun_out/r04n/c1.out"
