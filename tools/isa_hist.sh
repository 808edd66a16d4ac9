#!/bin/bash
# Instruction histogram of fd_dsm_kernel's inner doubling loop (gfx950 ISA).
# usage: tools/isa_hist.sh [extra hipcc flags...]   (writes /tmp/isa/dev.s)
set -e
mkdir -p /tmp/isa
SRC="$(dirname "$0")/../firedancer_amd/csrc/fd_ed25519_gpu.hip"
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/isa/dev.s "$@" "$SRC" 2>&1 | grep -i " error" || true
KN=${DSM_KERNEL:-fd_dsm_kernel}                     # fd_dsmh_kernel: the half-size walk
K=$(grep -o "^_Z${#KN}${KN}${DSM_INST:-ILi1E}[^:]*" /tmp/isa/dev.s | head -1)
awk -v k="$K:" 'index($0,k)==1{f=1} f{print} f&&/^\.Lfunc_end/{exit}' /tmp/isa/dev.s > /tmp/isa/dsm.s
L=$(grep -n "Inner Loop Header" /tmp/isa/dsm.s | head -1 | cut -d: -f1)
E=$(awk -v l="$L" 'NR>l && /s_cbranch_scc0/{print NR; exit}' /tmp/isa/dsm.s)
echo "doubling loop: lines $L-$E"
sed -n "${L},${E}p" /tmp/isa/dsm.s | grep -v "^\s*;" | grep -v "^\." | awk '{print $1}' | sort | uniq -c | sort -rn | head -20
echo "kernel VALU total: $(grep -c '^\s*v_' /tmp/isa/dsm.s)  s_nop: $(grep -c 's_nop' /tmp/isa/dsm.s)"
awk -v k="$K" 'index($0, ".name:") && index($0, k){f=1} f&&/\.vgpr_count/{print "vgpr " $2; exit}' /tmp/isa/dev.s
