#!/usr/bin/env python3
"""Reduce a rocprofv3 --kernel-trace CSV of the stream legs to per-queue facts about fd_gather_kernel:
its duration, the gap since the previous kernel ended on the same queue (back-to-back = it was queued
behind that one), how busy each queue was, and what else ran beside the gathers.

usage: trace_queue.py <dir with *kernel_trace.csv> [--drop]"""
import csv
import glob
import json
import os
import sys

import numpy as np


def pct(a):
    a = np.asarray(a, np.float64)
    if not len(a):
        return None
    return {k: round(float(np.percentile(a, p)), 1) for k, p in (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))}


def main():
    d = sys.argv[1]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            rows.append((r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"]), int(r.get("Queue_Id", 0) or 0), int(r.get("Grid_Size", 0) or 0)))
    rows.sort(key=lambda r: r[1])
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    out = {"span_s": (t1 - t0) * 1e-9, "queues": {}}
    byq = {}
    for r in rows:
        byq.setdefault(r[3], []).append(r)
    for q, rr in sorted(byq.items()):
        names = {}
        for r in rr:
            names[r[0]] = names.get(r[0], 0) + 1
        busy = sum(r[2] - r[1] for r in rr) / max(1, rr[-1][2] - rr[0][1])
        g = [(i, r) for i, r in enumerate(rr) if r[0] == "fd_gather_kernel"]
        info = {"kernels": names, "busy_frac": round(busy, 3)}
        if g:
            gaps = [(r[1] - rr[i - 1][2]) * 1e-3 for i, r in g if i > 0]
            info["gather_dur_us"] = pct([(r[2] - r[1]) * 1e-3 for _, r in g])
            info["gather_records"] = pct([r[4] / 64 for _, r in g])
            info["gather_gap_after_prev_us"] = pct(gaps)
            info["gather_back_to_back_frac"] = round(float(np.mean([x < 20 for x in gaps])) if gaps else 0.0, 3)
        out["queues"][q] = info
    # time-sliced view: per 0.25 s, gathers' total duration vs wall, and the number of other kernels running
    w = int(0.25e9)
    sl = []
    t = t0
    while t < t1:
        gd = sum(min(r[2], t + w) - max(r[1], t) for r in rows if r[0] == "fd_gather_kernel" and r[2] > t and r[1] < t + w)
        od = sum(min(r[2], t + w) - max(r[1], t) for r in rows if r[0] != "fd_gather_kernel" and r[2] > t and r[1] < t + w)
        sl.append({"t_s": round((t - t0) * 1e-9, 2), "gather_busy": round(gd / w, 2), "other_busy": round(od / w, 2)})
        t += w
    out["slices"] = sl
    json.dump(out, open(os.path.join(d, "queue_summary.json"), "w"), indent=1)
    print(json.dumps(out["queues"], indent=1))
    if "--drop" in sys.argv:
        os.unlink(kt)


if __name__ == "__main__":
    main()
