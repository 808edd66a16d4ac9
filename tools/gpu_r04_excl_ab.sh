#!/bin/bash
# Round 4 paced-leg A/B (the knee): latency-path workgroups alone on their CUs (--stream-cu-exclusive 1,
# fdgpu_ed25519_set_cu_exclusive), so the staggered batches of a tile's two contexts never share a SIMD.  First
# the engine-path parity tests on that path (latency8x) and the tile tests, then the tile process at 10M
# frags/s under a kernel trace, then interleaved legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
C="python3 bench.py --stream-child --stream-device 0 --stream-proc 0 --stream-procs 1 --stream-token pp --stream-seed 1234 --txns 65536 --stream-rates 10e6 --stream-only-paced --stream-paced-seconds 2"
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6,7.5e6,10e6,12.5e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04o/$1.json > gpurun_out/r04o/$1.out\""; }
eval bash tools/gpu_job.sh \
  "\"xtests:400:python -u -m pytest tests -m gpu -k 'latency8x or cu_split' -x -q --timeout 200 --timeout-method thread\"" \
  "\"xprof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/r04o/cx -o run -- $C --stream-cu-exclusive 1 > gpurun_out/r04o/cx.out\"" \
  "$(run e0a '')" "$(run e1a '--stream-cu-exclusive 1')" "$(run e1b '--stream-cu-exclusive 1')" "$(run e0b '')"
