#!/bin/bash
# tools/dispatchprobe: launch -> start delay of a small kernel / gather beside long verify-like kernels,
# one ingredient of the stream's GPU side at a time (flags: see the probe's header).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=gpurun_out/dispatch; mkdir -p $d
P=tools/dispatchprobe/dispatch_probe
specs=()
for f in ${DISPATCH_FLAGS:-i h gi gh gh_e gh_m gh_em g_em ghc_em}; do
  specs+=("$f:60:$P ${f//_/} ${DISPATCH_BLOCKS:-512} ${DISPATCH_US:-2000} ${DISPATCH_RECS:-1024} ${DISPATCH_DEPTH:-2} >> $d/probe.jsonl")
done
bash "$(dirname "$0")/gpu_job.sh" "${specs[@]}"
cat $d/probe.jsonl
