#!/bin/bash
# Build an engine variant for A/B runs: tools/ab_build.sh <name> [hipcc -D flags...]
# -> build/ab/<name>.so ; run with FDGPU_LIB=build/ab/<name>.so python bench.py ...
set -e
name="$1"; shift
cd "$(dirname "$0")/.."
mkdir -p build/ab
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function -Wno-unused-value -Wno-unused-result \
  -o "build/ab/$name.so" "$@" firedancer_amd/csrc/fd_ed25519_gpu.hip
echo "built build/ab/$name.so"
