#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --hip-runtime-trace run of the stream legs: for each kernel kind,
the delay from its launch call's return (HIP API trace, same Correlation_Id) to the kernel's start, and its
duration; fd_gather_kernel is the one that bounds a frag's exposure to a lapping producer.  Percentiles
over 0.5 s windows show how the delay moves with the load of each leg.

usage: trace_gather.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv> [--drop]"""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d = sys.argv[1]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    at = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    launch_end = {}
    with open(at) as f:
        for r in csv.DictReader(f):
            if "Launch" in r["Function"]:
                launch_end[r["Correlation_Id"]] = int(r["End_Timestamp"])
    rows = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            le = launch_end.get(r["Correlation_Id"])
            rows.append((name, s, e, (s - le) if le else None, int(r.get("Queue_Id", 0) or 0)))
    t0 = min(r[1] for r in rows)
    out = {"kernels": {}, "gather_windows": []}
    for name in sorted({r[0] for r in rows}):
        rr = [r for r in rows if r[0] == name]
        dl = np.array([r[3] for r in rr if r[3] is not None], np.float64) * 1e-3
        du = np.array([r[2] - r[1] for r in rr], np.float64) * 1e-3
        out["kernels"][name] = {"n": len(rr), "launch_to_start_us": {q: float(np.percentile(dl, p)) for q, p in
                                                                    (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))}
                                if len(dl) else None,
                                "dur_us": {"p50": float(np.percentile(du, 50)), "p99": float(np.percentile(du, 99))},
                                "queues": sorted({r[4] for r in rr})}
    g = sorted((r for r in rows if r[0] == "fd_gather_kernel" and r[3] is not None), key=lambda r: r[1])
    w = 0.5e9
    end = max(r[2] for r in rows)
    t = t0
    while t < end:
        x = [r for r in g if t <= r[1] < t + w]
        busy = sum(min(r[2], t + w) - max(r[1], t) for r in rows if r[0] != "fd_gather_kernel" and r[2] > t and r[1] < t + w)
        if x:
            dl = np.array([r[3] for r in x], np.float64) * 1e-3
            out["gather_windows"].append({"t_s": round((t - t0) * 1e-9, 2), "n": len(x), "delay_p50_us": float(np.median(dl)),
                                          "delay_p99_us": float(np.percentile(dl, 99)),
                                          "other_kernels_busy": round(busy / w, 2)})
        t += w
    json.dump(out, open(os.path.join(d, "gather_delay.json"), "w"), indent=1)
    print(json.dumps(out["kernels"].get("fd_gather_kernel"), indent=1))
    if "--drop" in sys.argv:
        for f in (kt, at):
            os.unlink(f)


if __name__ == "__main__":
    main()
