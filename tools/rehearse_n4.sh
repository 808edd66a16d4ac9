#!/bin/bash
# N=4 rehearsal of bench.py on a one-GPU box: four ranks on GPU 0 (FDGPU_BENCH_ONE_DEVICE=1), gloo
# collectives, four producer links and eight verify tiles in four processes sharing /dev/shm links.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
df -h /dev/shm
FDGPU_BENCH_ONE_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 4 --steps 3 --warmup 1 --txns 131072 --no-extra-configs --latency-batch 0 \
  --no-cpu-baseline --stream-seconds 2 --stream-unrel-seconds 1 "$@"
