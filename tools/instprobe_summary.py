#!/usr/bin/env python3
"""profiles/r03/roofline: tools/instprobe/instprobe2 under one PMC pass (GRBM_GUI_ACTIVE, SQ_INSTS_VALU,
SQ_WAVES, ...).  Per dispatch: the DVFS clock the guide prescribes (GRBM_GUI_ACTIVE / 8 XCDs / wall) and
the cycles per wave64 VALU instruction per SIMD it implies (wall x clock / (SQ_INSTS_VALU / 1024 SIMDs)),
next to the probe's own s_memtime-based figure.  usage: instprobe_summary.py <pmc csv> <probe.txt>"""
import collections
import csv
import sys

rows = collections.defaultdict(dict)
meta = {}
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        k = int(r["Dispatch_Id"])
        rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"].split("(")[0].replace("k_", ""), int(r["Grid_Size"]),
                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
probe = {}
with open(sys.argv[2]) as f:
    next(f)
    for line in f:
        p = line.split()
        if len(p) >= 7:
            probe.setdefault(p[0], []).append((int(p[1]), float(p[5]), float(p[3])))
agg = collections.defaultdict(list)
for k in sorted(rows):
    name, grid, dur = meta[k]
    c = rows[k]
    if "GRBM_GUI_ACTIVE" not in c or "SQ_INSTS_VALU" not in c or dur <= 0:
        continue
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9) / 1e6
    waves = c.get("SQ_WAVES", grid / 64)
    agg[(name, grid)].append((dur, clk, c["SQ_INSTS_VALU"] / max(waves, 1), dur * 1e-9 * clk * 1e6 / (c["SQ_INSTS_VALU"] / 1024)))
import statistics as stt
print(f"{'variant':16s} {'grid':>8s} {'n':>4s} {'wall_us':>8s} {'clk_MHz(GRBM)':>13s} {'VALU/wave':>10s} {'cyc/inst(PMC)':>13s}")
for (name, grid), v in agg.items():
    md = lambda i: stt.median(x[i] for x in v)
    print(f"{name:16s} {grid:8d} {len(v):4d} {md(0)*1e-3:8.1f} {md(1):13.0f} {md(2):10.0f} {md(3):13.2f}")
sys.exit(0)
seen = collections.Counter()
print(f"{'variant':16s} {'w/SIMD':>6s} {'wall_us':>8s} {'clk_MHz(GRBM)':>13s} {'VALU/wave':>10s} {'cyc/inst(PMC)':>13s} "
      f"{'cyc/inst(probe)':>15s} {'clk_MHz(probe)':>14s}")
for k in sorted(rows):
    name, grid, dur = meta[k]
    c = rows[k]
    if "GRBM_GUI_ACTIVE" not in c or "SQ_INSTS_VALU" not in c or dur <= 0:
        continue
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-9) / 1e6
    waves = c.get("SQ_WAVES", grid / 64)
    per_wave = c["SQ_INSTS_VALU"] / max(waves, 1)
    cyc = dur * 1e-9 * clk * 1e6 / (c["SQ_INSTS_VALU"] / 1024)
    i = seen[name]
    seen[name] += 1
    pr = probe.get(name, [])
    w, pc, pclk = pr[i] if i < len(pr) else (grid // (256 * 1024) * 4, float("nan"), float("nan"))
    print(f"{name:16s} {w:6d} {dur*1e-3:8.1f} {clk:13.0f} {per_wave:10.0f} {cyc:13.2f} {pc:15.2f} {pclk:14.0f}")
