#!/usr/bin/env python3
"""Summarise a tools/gpu_round.sh profile directory (rocprofv3 csv) into
per-kernel, per-launch numbers and write profiles/<round>/pmc_summary.json
(+ profiles/dsm_pmc.json, which bench.py reads for roofline.traffic).

Corrections (MI355X_MICROARCH.md, HBM section):
  * FETCH_SIZE / WRITE_SIZE are reported in KiB.
  * gfx950 FETCH_SIZE counts 128-B requests as 64 B for wide streaming
    reads: hbm_read_bytes = 2 x FETCH_SIZE x 1024 (an upper estimate for
    the DSM's 16-B-per-lane gathers, which are not calibrated).
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs; valu_busy_flat4 =
    SQ_ACTIVE_INST_VALU x 4 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) -- a
    flat 4-cycle price per instruction, kept for comparison with round 1.
    The measured-cost form is tools/dsm_issue_model.py (profiles/r02/
    roofline/issue_model.json), which dsm_pmc.json carries as valu_busy.
usage: tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>/<tag>
"""
import collections
import csv
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
# the 1M launch: the half-size walk (default), else the carry-folded full-length walk
DSM = ("fd_dsmh_kernel<1>", "fd_dsm_kernel<1>", "fd_dsm_kernel")


def norm(name):      # "void fd_dsm_kernel<1>(unsigned int, ...)" -> "fd_dsm_kernel<1>"
    n = name.split("(")[0].strip()
    return n[5:] if n.startswith("void ") else n


os.makedirs(dst, exist_ok=True)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("fetch", "write", "sq"):
    f = os.path.join(src, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        per[norm(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, c in per.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    e = {"launches_sampled": max(len(v) for v in c.values()), "counters_mean_per_launch": m}
    if "FETCH_SIZE" in m:
        e["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        e["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_ACTIVE_INST_VALU" in m and m.get("GRBM_GUI_ACTIVE"):
        e["valu_busy_flat4"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
        e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    out[k] = e
json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
stats = os.path.join(src, "stats", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
# the bench line printed by the profiled run itself: its HIP-event kernel_ms must agree with
# rocprof's average duration of the same launches
blog = os.path.join(src, "bench_under_rocprof.log")
if not os.path.exists(blog):
    blog = os.path.join(src, "bench_under_rocprof.json")
if os.path.exists(blog):
    for line in open(blog):
        if line.startswith('{"metric"'):
            b = json.loads(line)
            agree = {"bench_hip_event_dsm_ms": b["kernel_ms"]["dsm"]}
            if os.path.exists(stats):
                for r in csv.DictReader(open(stats)):
                    if norm(r["Name"]) in DSM:
                        agree["rocprof_avg_dsm_ms"] = float(r["AverageNs"]) / 1e6
                        agree["rocprof_calls"] = int(r["Calls"])
            b["rocprof_agreement"] = agree
            json.dump(b, open(os.path.join(dst, "bench_under_rocprof.json"), "w"), indent=1)
            print("agreement", agree)
dk = next((k for k in DSM if k in out), None)
d = out.get(dk)
if d and "hbm_read_bytes" in d:
    rd = os.path.join(os.path.dirname(dst.rstrip("/")), "roofline")
    im = os.path.join(rd, "issue_model_dsmh_r03c.json")      # the model priced with every measured row
    if dk.startswith("fd_dsmh") and not os.path.exists(im):  # a later round without its own model: the last one
        im = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r03", "roofline",
                          "issue_model_dsmh_r03c.json")
    if not dk.startswith("fd_dsmh") or not os.path.exists(im):
        im = os.path.join(rd, "issue_model_dsmh.json" if dk.startswith("fd_dsmh") else "issue_model.json")
    busy = None
    if os.path.exists(im):
        mj = json.load(open(im))
        busy = mj["valu_busy_model"]
        # the model's issue time (at its clock) over THIS run's measured launch time, when rocprof has it
        for r in (csv.DictReader(open(stats)) if os.path.exists(stats) else []):
            if norm(r["Name"]) == dk and mj.get("predicted_ms"):
                busy = mj["predicted_ms"] / (float(r["AverageNs"]) / 1e6)
    json.dump({"kernel": dk, "source": dst,
               "hbm_bytes_per_launch": d["hbm_read_bytes"] + d.get("hbm_write_bytes", 0),
               "valu_busy": busy,
               "valu_busy_source": os.path.relpath(os.path.abspath(im), os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
                                   + " (predicted issue time / this run's rocprof launch time)" if busy is not None else None,
               "valu_busy_flat4": d.get("valu_busy_flat4"), "valu_insts_per_wave": d.get("valu_insts_per_wave"),
               # the throughput path's other big kernels, per 1M-sig launch: the decode kernel writes the -A / -R
               # tables (per signature, HBM-resident) that the walk reads; the hash kernel reads the messages
               "per_kernel": {k: {"hbm_read_bytes": out[k].get("hbm_read_bytes"), "hbm_write_bytes": out[k].get("hbm_write_bytes"),
                                  "valu_busy_flat4": out[k].get("valu_busy_flat4"),
                                  "valu_insts_per_wave": out[k].get("valu_insts_per_wave")}
                              for k in (dk, "fd_decode_kernel", "fd_hashh_kernel") if k in out}},
              open(os.path.join(os.path.dirname(dst.rstrip("/")), "..", "dsm_pmc.json"), "w"), indent=1)
for k, e in sorted(out.items()):
    print(k, {x: (round(y, 3) if isinstance(y, float) else y) for x, y in e.items() if x != "counters_mean_per_launch"})
