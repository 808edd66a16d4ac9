#!/bin/bash
# round 3: paced-latency A/B (the knee): contexts per tile, tiles, copy wait
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_BASE="--stream-procs 1 --stream-seconds 1 --stream-paced-seconds 3 --stream-unrel-seconds 1 --stream-rates 2e6,5e6" \
bash tools/gpu_stream_ab.sh lat "" "--stream-lat-ctx 3" "--stream-lat-tiles 3" "--stream-lat-tiles 3 --stream-lat-ctx 3" "--stream-copy-wait-us 20" "--stream-lat-tiles 1 --stream-lat-ctx 3"
