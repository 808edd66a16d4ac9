#!/usr/bin/env python3
"""Reduce a rocprofv3 --kernel-trace CSV of paced stream legs to the batch chain's parts: per kernel, its
duration; per consecutive pair on one queue, the gap between the first's end and the second's start (the
dispatch of a dependent kernel; gaps over 1 ms, a queue idle between batches, are left out); and per batch,
its whole chain on its queue: fd_parse_kernel's start to the next fd_done_kernel's end.

usage: trace_chain.py <dir with *kernel_trace.csv>"""
import collections
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
    return {"n": int(len(a)), **{k: round(float(np.percentile(a, p)), 1) for k, p in (("p50", 50), ("p90", 90), ("p99", 99))}}


def main():
    kt = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    q = collections.defaultdict(list)
    with open(kt) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            q[int(r.get("Queue_Id", 0) or 0)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    dur, gap, chain = collections.defaultdict(list), collections.defaultdict(list), []
    for ks in q.values():
        ks.sort()
        t0 = None
        for s, e, n in ks:
            if n == "fd_parse_kernel":
                t0 = s
            elif n == "fd_done_kernel" and t0 is not None:
                chain.append((e - t0) / 1e3)
                t0 = None
        for i, (s, e, n) in enumerate(ks):
            dur[n].append((e - s) / 1e3)
            if i:
                ps, pe, pn = ks[i - 1]
                g = (s - pe) / 1e3
                if 0 <= g < 1000:
                    gap[f"{pn} -> {n}"].append(g)
    print(json.dumps({"chain_us": pct(chain), "duration_us": {k: pct(v) for k, v in sorted(dur.items())},
                      "gap_us": {k: pct(v) for k, v in sorted(gap.items()) if len(v) > 20}}, indent=1))


if __name__ == "__main__":
    main()
