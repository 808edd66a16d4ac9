#!/bin/bash
# Round 4: multi-rank rehearsals of the final build on a one-GPU box (every rank on GPU 0): N=2 under
# torch.distributed.run (the driver's launch) and N=4 through bench.py's own launcher.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04t
bash tools/gpu_job.sh \
  "n2:400:bash tools/rehearse_n2.sh --stream-rates 2e6,4e6 --stream-paced-seconds 2 --detail-out gpurun_out/r04t/n2.json > gpurun_out/r04t/n2.out" \
  "n4:400:FDGPU_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 4 --steps 3 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 1e6,2e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --detail-out gpurun_out/r04t/n4.json > gpurun_out/r04t/n4.out"
