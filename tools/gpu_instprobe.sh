#!/bin/bash
# VALU issue-rate evidence (profiles/r03/roofline): tools/instprobe/instprobe2 plain, under a kernel
# trace (durations), under one PMC pass (GRBM_GUI_ACTIVE for the DVFS clock, SQ instruction and cycle
# counters), and the gfx950 counter list.
# usage: gpurun --timeout 600 -- 'bash tools/gpu_instprobe.sh'
d=gpurun_out/instprobe
mkdir -p $d
P=tools/instprobe/instprobe2
bash "$(dirname "$0")/gpu_job.sh" \
  "probe:120:$P 2048 > $d/probe.txt" \
  "probe_stats:120:rocprofv3 --kernel-trace --stats -f csv -d $d/stats -o run -- $P 2048 > $d/probe_under_trace.txt" \
  "probe_pmc:120:timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -f csv -d $d/pmc -o run -- $P 2048 > $d/probe_under_pmc.txt" \
  "counters:60:timeout -s KILL 50 rocprofv3 -L > $d/counters.txt 2>&1"
