#!/bin/bash
# Round 4 stream A/B on a quiet box, interleaved: the gather path.  The GPU reads every record over PCIe through
# the IOMMU; a 4 KiB-page link region costs an IOTLB (and a host dTLB) miss per record.  Arms: the default;
# the link in transparent huge pages (--stream-huge); 4 records per gather workgroup; 32 gather CUs; huge + 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04i
(cat /sys/kernel/mm/transparent_hugepage/enabled /sys/devices/system/clocksource/clocksource0/current_clocksource;
 for g in /sys/kernel/iommu_groups/*; do t=$(cat $g/type 2>/dev/null); echo "$(basename $g) $t $(ls $g/devices | head -3 | tr '\n' ' ')"; done | awk '{print $2}' | sort | uniq -c;
 python3 -c "import ctypes; print('ok')") > gpurun_out/r04i/sysinfo.txt 2>&1
S="python3 bench.py --steps 2 --warmup 1 --txns 262144 --no-cpu-baseline --no-extra-configs --latency-batch 0 --stream-rates 7.5e6,10e6 --stream-paced-seconds 2 --stream-seconds 5 --stream-unrel-seconds 1 --stream-prof"
run() { echo "\"$1:200:$S $2 --detail-out gpurun_out/r04i/$1.json > gpurun_out/r04i/$1.out\""; }
eval bash tools/gpu_job.sh \
  "$(run base1 '')" "$(run huge1 '--stream-huge')" "$(run rpb4a '--stream-gather-rpb 4')" \
  "$(run cu32a '--stream-gather-cus 32')" "$(run hr4a '--stream-huge --stream-gather-rpb 4')" \
  "$(run hr4b '--stream-huge --stream-gather-rpb 4')" "$(run cu32b '--stream-gather-cus 32')" \
  "$(run rpb4b '--stream-gather-rpb 4')" "$(run huge2 '--stream-huge')" "$(run base2 '')"
