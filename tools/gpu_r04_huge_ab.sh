#!/bin/bash
# Round 4 stream A/B on one box, interleaved (ABCDDCBA): the default build (link in 4 KiB pages, 1 record
# per gather workgroup, as validated in round 3), 4 records per gather workgroup (--stream-gather-rpb 4), the
# link in transparent huge pages (--stream-huge), the stream legs before the bench process initialises the GPU (--stream-first), and
# 65,536 instead of 16,384 frags a tile may hold uncopied (--stream-max-uncopied), with copies started after
# 200 instead of 50 us (bigger gathers: round 2's probe moved 30 GB/s at 4,096 records, 36-41 at 16-64K).
# First the vtile / stream-parity GPU tests (the gather kernel changed); last an N=4 rehearsal of the
# self-launching bench with every rank on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04g
(cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled; cat /proc/cmdline;
 ls /sys/class/iommu 2>&1; ls /sys/kernel/iommu_groups 2>/dev/null | wc -l; grep -i huge /proc/meminfo) > gpurun_out/r04g/sysinfo.txt 2>&1
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04g/$1.json > gpurun_out/r04g/$1.out\""; }
eval bash tools/gpu_job.sh \
  "\"vt:400:python -u -m pytest tests/test_gpu_vtile.py tests/test_gpu_faults.py tests/test_gpu_stream_parity.py -x -q --timeout 200 --timeout-method thread\"" \
  "$(run base1 '')" "$(run cw200a '--stream-copy-wait-us 200 --stream-max-uncopied 65536')" "$(run rpb4a '--stream-gather-rpb 4')" \
  "$(run huge1 '--stream-huge')" "$(run first1 '--stream-first')" "$(run unc64a '--stream-max-uncopied 65536')" \
  "$(run unc64b '--stream-max-uncopied 65536')" "$(run first2 '--stream-first')" "$(run huge2 '--stream-huge')" \
  "$(run rpb4b '--stream-gather-rpb 4')" "$(run cw200b '--stream-copy-wait-us 200 --stream-max-uncopied 65536')" "$(run base2 '')" \
  "\"n4:400:FDGPU_BENCH_ONE_DEVICE=1 python3 bench.py --gpus 4 --steps 3 --warmup 1 --txns 262144 --no-cpu-baseline --stream-rates 1e6,2e6 --stream-paced-seconds 2 --stream-seconds 3 --stream-unrel-seconds 1 --detail-out gpurun_out/r04g/n4.json > gpurun_out/r04g/n4.out\""
