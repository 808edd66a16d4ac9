#!/bin/bash
# The GPU verify tile under seccomp (tools/sandbox/vtile_sandbox.c): discover the syscalls a tile makes after
# its privileged init, then enforce exactly the policy in firedancer_amd/fd_verify_gpu_tile.seccomppolicy.
# usage: gpurun --timeout 300 -- 'bash tools/gpu_sandbox.sh'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
d=gpurun_out/sandbox
mkdir -p $d
# the syscall names of the policy file: lines "name" or "name: (...)" outside comments
allow=$(python3 -c "
import re
names=[]
for l in open('firedancer_amd/fd_verify_gpu_tile.seccomppolicy'):
    m=re.match(r'^([a-z_0-9]+)\s*(:|$)', l)
    if m and not l.startswith('unsigned'): names.append(m.group(1))
print(' '.join(names))")
echo "policy: $allow" > $d/policy_names.txt
bash "$(dirname "$0")/gpu_job.sh" \
  "discover:120:tools/sandbox/vtile_sandbox discover > $d/discover.json" \
  "enforce:120:tools/sandbox/vtile_sandbox enforce $allow > $d/enforce.json"
cat $d/discover.json $d/enforce.json
