#!/bin/bash
# Completion-poll software prefetch A/B (max-rate, unreliable and paced legs), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_BASE="--stream-procs 1 --stream-seconds 3 --stream-paced-seconds 2 --stream-unrel-seconds 2 --stream-rates 7.5e6" \
  bash tools/gpu_stream_ab.sh pollpf "" "--stream-poll-prefetch 16" "--stream-poll-prefetch 64" "" "--stream-poll-prefetch 16" "--stream-poll-prefetch 64"
