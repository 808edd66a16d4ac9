#!/bin/bash
# one async raw batch's latency and its kernels (tools/raw_batch_probe.py), plain and under a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=gpurun_out/rawprobe; mkdir -p $d
bash tools/gpu_job.sh \
  "raw:200:python tools/raw_batch_probe.py 512 1536 4096 > $d/plain.jsonl" \
  "raw_trace:300:rocprofv3 --kernel-trace --stats -f csv -d $d/t -o run -- python3 tools/raw_batch_probe.py 1536 > $d/traced.jsonl"
cat $d/plain.jsonl $d/traced.jsonl
