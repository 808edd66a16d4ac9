#!/bin/bash
# Round 4 stream A/B: the link region in transparent huge pages (default) vs 4 KiB pages (--stream-no-huge),
# and the stream legs run before the bench process initialises the GPU (--stream-first); then an N=4
# rehearsal of the self-launching bench with every rank on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04g
(cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled; cat /proc/cmdline;
 ls /sys/class/iommu 2>&1; ls /sys/kernel/iommu_groups 2>/dev/null | wc -l; grep -i huge /proc/meminfo) > gpurun_out/r04g/sysinfo.txt 2>&1
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
bash tools/gpu_job.sh \
  "huge1:200:$S --detail-out gpurun_out/r04g/huge1.json > gpurun_out/r04g/huge1.out" \
  "small1:200:$S --stream-no-huge --detail-out gpurun_out/r04g/small1.json > gpurun_out/r04g/small1.out" \
  "first1:200:$S --stream-first --detail-out gpurun_out/r04g/first1.json > gpurun_out/r04g/first1.out" \
  "first2:200:$S --stream-first --detail-out gpurun_out/r04g/first2.json > gpurun_out/r04g/first2.out" \
  "small2:200:$S --stream-no-huge --detail-out gpurun_out/r04g/small2.json > gpurun_out/r04g/small2.out" \
  "huge2:200:$S --detail-out gpurun_out/r04g/huge2.json > gpurun_out/r04g/huge2.out" \
  "n4:400:FDGPU_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 4 --steps 3 --warmup 1 --txns 262144 --no-cpu-baseline --stream-rates 1e6,2e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --detail-out gpurun_out/r04g/n4.json > gpurun_out/r04g/n4.out"
