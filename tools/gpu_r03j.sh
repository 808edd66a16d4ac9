#!/bin/bash
# Paced legs: engine contexts per tile (2 = default, 3, 4) and 2 tiles, at 7.5 / 10 / 12.5M frags/s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_BASE="--stream-procs 1 --stream-seconds 1 --stream-paced-seconds 3 --stream-unrel-seconds 1 --stream-rates 7.5e6,10e6,12.5e6" \
  bash tools/gpu_stream_ab.sh latctx "--stream-lat-ctx 2" "--stream-lat-ctx 3" "--stream-lat-ctx 4" "--stream-lat-ctx 2 --stream-lat-tiles 2" "--stream-lat-ctx 3" "--stream-lat-ctx 2"
