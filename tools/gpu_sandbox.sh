#!/bin/bash
# The verify tile under seccomp (tools/sandbox/vtile_sandbox.c), round 6: the tile with its own GPU context at the
# bench's paced defaults (two contexts, exclusive CUs within their shares, 16 copy CUs), without and with its launch
# thread -- discover the syscalls it makes after privileged init, then enforce exactly
# firedancer_amd/fd_verify_gpu_tile.seccomppolicy -- and the served form: a tile process without a GPU context
# enforced under the reference verify tile's own policy (write, fsync: src/disco/verify/fd_verify_tile.seccomppolicy)
# beside its verify service (discovered, then enforced under firedancer_amd/fd_verify_service.seccomppolicy).
# usage: gpurun --timeout 400 -- 'bash tools/gpu_sandbox.sh [outdir]'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=${1:-gpurun_out/sandbox}
mkdir -p $d
names() { python3 -c "
import re,sys
names=[]
for l in open(sys.argv[1]):
    m=re.match(r'^([a-z_0-9]+)\s*(:|$)', l)
    if m and not l.startswith('unsigned'): names.append(m.group(1))
print(' '.join(names))" "$1"; }
tile=$(names firedancer_amd/fd_verify_gpu_tile.seccomppolicy)
svc=$(names firedancer_amd/fd_verify_service.seccomppolicy)
echo "tile policy: $tile / service policy: $svc" > $d/policy_names.txt
S=tools/sandbox/vtile_sandbox
bash "$(dirname "$0")/gpu_job.sh" \
  "discover:120:$S discover > $d/discover.json" \
  "enforce:120:$S enforce $tile > $d/enforce.json" \
  "discover_launcher:120:$S discover --launcher > $d/discover_launcher.json" \
  "enforce_launcher:120:$S enforce --launcher $tile > $d/enforce_launcher.json" \
  "served_discover:120:$S served discover --launcher > $d/served_discover.json" \
  "served_enforce:120:$S served enforce --launcher write fsync -- $svc > $d/served_enforce.json"
cat $d/*.json
