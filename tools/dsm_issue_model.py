#!/usr/bin/env python3
"""Issue-cost model of fd_dsm_kernel from its gfx950 ISA and measured per-instruction costs.

1. The kernel's basic blocks (tools/isa_hist.sh writes /tmp/isa/dsm.s) are weighted by how often one
   signature executes them: the loop structure of fd_dsm_kernel (64 windows: 63 x 3 inner doublings
   to P2, 63 doublings to P3, 64 -A table adds, 16 base-point adds, 64 P2 conversions, 16 base-point
   gathers, the prologue and the deferred-R epilogue once).  The weighted VALU count is checked
   against the PMC SQ_INSTS_VALU per wave (profiles: 338,222 in round 1).
2. Each VALU mnemonic is priced at the cycles per wave64 instruction per SIMD that tools/instprobe
   measured on MI355X (16 independent chains, 8 waves per SIMD, shader clock from s_memtime /
   s_memrealtime); s_nop is priced at 0 (another wave issues meanwhile).
3. Predicted kernel time = waves per SIMD x (issue cycles per wave) / clock, against the measured
   fd_dsm_kernel time: their ratio is the VALU busy fraction under the measured costs.

usage: dsm_issue_model.py instprobe.log --dsm-ms 9.57 --clock-mhz 2350 [--asm /tmp/isa/dsm.s] [--nsig 1048576]
       [--kernel dsmh]   (the half-size walk: DSM_KERNEL=fd_dsmh_kernel tools/isa_hist.sh first)
"""
import argparse
import json
import re
import sys

# weights of the blocks of the current fd_dsm_kernel build, in order (see the docstring); the model
# refuses an ISA whose block count or VALU total does not match (rebuild the weights then)
BLOCK_WEIGHTS = [("start", 0), ("bb0", 1), ("bb1", 1), ("bb2 prologue", 1), ("window header + -A gather", 64),
                 ("w==63 skip", 1), ("base-point gather", 16), ("inner header", 63),
                 ("inner loop: dbl -> P2", 189), ("dbl -> P3", 63), ("-A table add", 64), ("base-point add", 16),
                 ("-> P2", 64), ("next digit", 63), ("loop tail", 64), ("back edge", 64), ("exit", 1),
                 ("deferred-R store", 1), ("R compare (latency builds only)", 0), ("ret", 1), ("ret2", 1)]

# fd_dsmh_kernel<1> (the half-size walk, wtop = 32: 33 windows, 32 with doublings, 16 base-point windows;
# tools/isa_hist.sh with DSM_KERNEL=fd_dsmh_kernel); blocks 40-56 are the slow-list role (dsm_one), 0 here
HS_BLOCK_WEIGHTS = ([(f"prologue {i}", 1) for i in range(26)] +
                    [("walk prologue", 1), ("loop latch", 32), ("window header + -A gather", 33), ("dbl entry", 32),
                     ("inner loop: dbl -> P2", 96), ("dbl -> P3", 32), ("-A add -> P3, -R gather", 33),
                     ("base-point digit", 16), ("-R add", 33), ("base-point add", 16), ("-> P2, next", 33),
                     ("digit loads", 32), ("identity check", 1), ("exit", 1)] +
                    [(f"slow role {i}", 0) for i in range(19)])

# instprobe row for each mnemonic family
ROW = {"v_mad_u64_u32": "v_mad_u64_u32", "v_and_b32": "v_and_b32", "v_lshrrev_b64": "v_lshrrev_b64",
       "v_lshlrev_b32": "v_lshlrev_b32", "v_add_u32": "v_add_u32", "v_mul_lo_u32": "v_mul_lo_u32",
       "v_lshl_add_u64": "v_lshl_add_u64", "v_sub_u32": "v_sub_u32", "v_alignbit_b32": "v_alignbit_b32",
       "v_mov_b32": "v_mov_b32", "v_mad_u32_u24": "v_mad_u32_u24", "v_lshrrev_b32": "v_lshrrev_b32",
       "v_cndmask_b32": "v_cmp+v_cndmask", "v_lshl_add_u32": "v_lshl_add_u32", "v_bitop3_b32": "v_bitop3_b32",
       "v_mul_u32_u24": "v_mul_u32_u24", "v_or_b32": "v_and_b32", "v_xor_b32": "v_and_b32",
       "v_subrev_u32": "v_sub_u32", "v_add_co_u32": "v_add_co_u32", "v_addc_co_u32": "v_add_co_u32",
       "v_cmp_gt_i32": "v_add_u32", "v_cmp_lt_i32": "v_add_u32", "v_cmp_eq_u32": "v_add_u32",
       "v_cmp_ne_u32": "v_add_u32", "v_ashrrev_i32": "v_lshrrev_b32", "v_bfe_u32": "v_alignbit_b32",
       "v_readfirstlane_b32": "v_mov_b32", "v_lshl_or_b32": "v_lshl_or_b32", "v_and_or_b32": "v_add3_u32",
       "v_add3_u32": "v_add3_u32", "v_or3_b32": "v_add3_u32", "v_max_i32": "v_add_u32",
       "v_sub_co_u32": "v_add_co_u32", "v_subb_co_u32": "v_add_co_u32", "v_ashrrev_i64": "v_lshrrev_b64",
       "v_lshlrev_b64": "v_lshrrev_b64", "v_mul_hi_u32": "v_mul_lo_u32", "v_bfi_b32": "v_bfi_b32",
       "v_perm_b32": "v_perm_b32", "v_alignbyte_b32": "v_alignbit_b32"}


def parse_probe(path):
    cyc = {}
    for line in open(path):
        m = re.match(r"^(\S.*?)\s{2,}([\d.]+)\s+(\d+)\s+([\d.]+)\s+([\d.]+)\s*$", line.rstrip())
        if m:
            cyc[m.group(1).strip()] = float(m.group(4))
    return cyc


def blocks_of(asm_path):
    lines = open(asm_path).read().split("\n")
    blocks, cur = [], None
    for l in lines:
        m = re.match(r"^(\.LBB\d+_\d+):|^; (%bb\.\d+):", l)
        if m:
            cur = {}
            blocks.append(cur)
            continue
        if cur is None:
            cur = {}
            blocks.append(cur)
        t = l.strip().split()
        if t and (t[0].startswith("v_") or t[0] == "s_nop"):
            k = re.sub(r"_e(32|64)$", "", t[0])
            cur[k] = cur.get(k, 0) + 1
    return blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("probe")
    ap.add_argument("--asm", default="/tmp/isa/dsm.s")
    ap.add_argument("--dsm-ms", type=float, required=True)
    ap.add_argument("--clock-mhz", type=float, required=True)
    ap.add_argument("--nsig", type=int, default=1 << 20)
    ap.add_argument("--pmc-valu-per-wave", type=float, default=338222.0)
    ap.add_argument("--kernel", choices=("dsm", "dsmh"), default="dsm")
    a = ap.parse_args()
    weights = HS_BLOCK_WEIGHTS if a.kernel == "dsmh" else BLOCK_WEIGHTS
    cyc = parse_probe(a.probe)
    blocks = blocks_of(a.asm)
    if len(blocks) != len(weights):
        sys.exit(f"ISA has {len(blocks)} blocks, the weights describe {len(weights)}: re-derive the weights")
    mix = {}
    for (name, w), b in zip(weights, blocks):
        for k, c in b.items():
            mix[k] = mix.get(k, 0) + w * c
    valu = sum(c for k, c in mix.items() if k.startswith("v_"))
    cost, unpriced = 0.0, {}
    by = {}
    for k, c in mix.items():
        if k == "s_nop":
            continue
        row = ROW.get(k)
        if row is None or row not in cyc:
            unpriced[k] = c
            row_c = cyc.get("v_add_u32", 3.0)
        else:
            row_c = cyc[row]
        cost += c * row_c
        by[k] = (c, row_c, c * row_c)
    waves_per_simd = a.nsig / 64 / 1024
    pred_ms = waves_per_simd * cost / (a.clock_mhz * 1e3)
    out = {"valu_per_wave_model": valu, "valu_per_wave_pmc": a.pmc_valu_per_wave,
           "s_nop_per_wave": mix.get("s_nop", 0), "issue_cycles_per_wave": cost,
           "waves_per_simd": waves_per_simd, "clock_mhz": a.clock_mhz, "predicted_ms": pred_ms,
           "measured_ms": a.dsm_ms, "valu_busy_model": pred_ms / a.dsm_ms,
           "mad_share_of_cycles": by.get("v_mad_u64_u32", (0, 0, 0))[2] / cost,
           "unpriced_mnemonics (priced as v_add_u32)": unpriced,
           "mix": {k: {"count": v[0], "cyc": v[1], "cycles": round(v[2])}
                   for k, v in sorted(by.items(), key=lambda kv: -kv[1][2])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
