#!/bin/bash
# Round 4: request sizes of the PCIe gather (tools/gatherprobe: the engine's record gather and a DMA of the same
# bytes), two PMC passes of TCC fabric request counters, plus one plain run for the GB/s table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
bash tools/gpu_job.sh \
  "gp:120:tools/gatherprobe/gather_probe > gpurun_out/r04v/probe.log" \
  "gpr:90:timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -f csv -d gpurun_out/r04v/rd -o run -- tools/gatherprobe/gather_probe" \
  "gpw:90:timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -f csv -d gpurun_out/r04v/wr -o run -- tools/gatherprobe/gather_probe"
