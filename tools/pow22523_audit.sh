#!/bin/bash
# fe_pow22523's squaring in fd_decode_kernel: the gfx950 ISA of each fe_sqn loop body (one
# squaring per trip) as an instruction histogram, and the decode kernel's VALU per wave from the committed PMC.
# usage: tools/pow22523_audit.sh [out]     (CPU only: hipcc cross-compiles; default out profiles/r06/pow22523_audit.txt)
set -e
cd "$(dirname "$0")/.."
out=${1:-profiles/r06/pow22523_audit.txt}
mkdir -p /tmp/isa "$(dirname "$out")"
hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/isa/dev.s \
  firedancer_amd/csrc/fd_ed25519_gpu.hip 2>&1 | grep -i " error" || true
K=$(grep -o "^_Z16fd_decode_kernel[^:]*" /tmp/isa/dev.s | head -1)
awk -v k="$K:" 'index($0,k)==1{f=1} f{print} f&&/^\.Lfunc_end/{exit}' /tmp/isa/dev.s > /tmp/isa/dec.s
{
  echo "fd_decode_kernel ($K): fe_sqn loop bodies (one fe_sqr per trip)"
  grep -n "Inner Loop Header" /tmp/isa/dec.s | cut -d: -f1 | while read L; do
    E=$(awk -v l="$L" 'NR>l && /s_cbranch_scc1/{print NR; exit}' /tmp/isa/dec.s)
    n=$(sed -n "${L},${E}p" /tmp/isa/dec.s | grep -c "^\s*v_")
    m=$(sed -n "${L},${E}p" /tmp/isa/dec.s | grep -c "^\s*v_mad_u64_u32")
    echo "loop at line $L: $n VALU, $m v_mad_u64_u32"
  done
  L=$(grep -n "Inner Loop Header" /tmp/isa/dec.s | head -1 | cut -d: -f1)
  E=$(awk -v l="$L" 'NR>l && /s_cbranch_scc1/{print NR; exit}' /tmp/isa/dec.s)
  echo "first loop body, by opcode:"
  sed -n "${L},${E}p" /tmp/isa/dec.s | grep -v "^\s*;" | grep -v "^\." | awk '{print $1}' | sort | uniq -c | sort -rn
  python3 - <<'EOF'
import json
pm = json.load(open("profiles/dsm_pmc.json"))
e = (pm.get("per_kernel") or {}).get("fd_decode_kernel") or {}
print("PMC fd_decode_kernel VALU per wave:", e.get("valu_insts_per_wave"), "(profiles/dsm_pmc.json)")
EOF
} > "$out"
cat "$out"
