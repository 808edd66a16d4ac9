#!/bin/bash
# round 3: stream tiles / gather-CU / copy-backlog A/B with the write-back (valid configurations), and the
# sandbox enforce run of the trimmed policy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_sandbox.sh
AB_BASE="--stream-procs 1 --stream-seconds 4 --stream-paced-seconds 3 --stream-unrel-seconds 2 --stream-rates 2e6,10e6,15e6" \
bash tools/gpu_stream_ab.sh tiles "--stream-gather-cus 16" "--stream-gather-cus 0" "--stream-gather-cus 16 --stream-tiles 3" "--stream-gather-cus 16 --stream-tiles 4" "--stream-gather-cus 16 --stream-max-uncopied 32768" "--stream-gather-cus 32 --stream-tiles 3"
