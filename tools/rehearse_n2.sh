#!/bin/bash
# N=2 rehearsal of bench.py on a one-GPU box: both ranks on GPU 0 (FDGPU_BENCH_ONE_DEVICE=1), gloo
# collectives, the configs[4] link shared through /dev/shm between the two ranks' tile processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
FDGPU_BENCH_ONE_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --txns 262144 --no-extra-configs --latency-batch 0 \
  --stream-seconds 3 --stream-unrel-seconds 2 "$@"
