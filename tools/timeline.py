#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 --kernel-trace (+ --memory-copy-trace) CSV of a stream run.

Per kernel: calls, mean duration; over the traced window: how much of the wall time had >= 1
kernel running (device busy), the mean number of concurrent kernels, the busy time of each kernel
family, the gap between consecutive kernels of one queue, and per-batch chain length (gather ->
done kernel on one queue).

usage: timeline.py <dir with *_kernel_trace.csv> [--skip-ms 300]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name):
    return name.split("(")[0].split("<")[0]


def load(path, pattern):
    rows = []
    for f in glob.glob(os.path.join(path, "**", pattern), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip-ms", type=float, default=300.0, help="ignore the first ms of the trace (setup)")
    a = ap.parse_args()
    ks = load(a.dir, "*kernel_trace.csv")
    cs = load(a.dir, "*memory_copy_trace.csv")
    ev = []
    for r in ks:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?")))
    for r in cs:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy_" + r.get("Direction", "?"), "dma"))
    ev.sort()
    t0 = ev[0][0] + int(a.skip_ms * 1e6)
    # window: from t0 to the last fd_done_kernel
    ev = [e for e in ev if e[0] >= t0 and not e[2].startswith("fd_btab")]
    t_end = max(e[1] for e in ev)
    wall = t_end - t0
    fam = defaultdict(lambda: [0, 0])
    for s, e, n, q in ev:
        fam[n][0] += 1
        fam[n][1] += e - s
    # union busy and concurrency of kernels (copies separately)
    def union(es):
        pts = sorted([(s, 1) for s, e, *_ in es] + [(e, -1) for s, e, *_ in es])
        busy, cur, last, area = 0, 0, None, 0
        for t, d in pts:
            if last is not None and cur > 0:
                busy += t - last
                area += cur * (t - last)
            cur += d
            last = t
        return busy, area
    kev = [e for e in ev if not e[2].startswith("copy_")]
    cev = [e for e in ev if e[2].startswith("copy_")]
    kb, ka = union(kev)
    cb, _ = union(cev) if cev else (0, 0)
    dsm = [e for e in kev if e[2].startswith("fd_dsm")]
    db, da = union(dsm)
    gat = [e for e in kev if e[2] == "fd_gather_kernel"]
    gb, ga = union(gat)
    out = {"window_ms": wall / 1e6, "kernels": len(kev), "copies": len(cev),
           "kernel_busy_frac": kb / wall, "kernel_mean_concurrency_when_busy": ka / max(kb, 1),
           "copy_busy_frac": cb / wall, "dsm_busy_frac": db / wall, "dsm_mean_concurrency": da / max(db, 1),
           "gather_busy_frac": gb / wall, "gather_mean_concurrency": ga / max(gb, 1),
           "families": {n: {"calls": c, "mean_us": round(t / c / 1e3, 1), "sum_ms": round(t / 1e6, 1),
                            "sum_frac_of_wall": round(t / wall, 3)}
                        for n, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1])}}
    # per queue: chain from fd_gather_kernel to the next fd_done_kernel, and idle gaps
    byq = defaultdict(list)
    for e in kev:
        byq[e[3]].append(e)
    chains, gaps = [], []
    for q, es in byq.items():
        es.sort()
        start = None
        for i, (s, e, n, _) in enumerate(es):
            if i:
                gaps.append(s - es[i - 1][1])
            if n in ("fd_gather_kernel", "fd_parse_kernel") and start is None:
                start = s
            if n == "fd_done_kernel" and start is not None:
                chains.append(e - start)
                start = None
    chains.sort()
    gaps.sort()
    if chains:
        out["batch_chain_us"] = {"n": len(chains), "p50": chains[len(chains) // 2] / 1e3,
                                 "p90": chains[int(len(chains) * .9)] / 1e3}
    if gaps:
        out["queue_gap_us"] = {"p50": gaps[len(gaps) // 2] / 1e3, "p90": gaps[int(len(gaps) * .9)] / 1e3,
                               "sum_ms": sum(gaps) / 1e6}
    out["queues"] = len(byq)
    # which kernel families run beside a DSM kernel, as a fraction of the DSM's time
    qstream = defaultdict(set)
    for r in ks:
        qstream[r.get("Queue_Id", "?")].add(r.get("Stream_Id", "?"))
    out["streams_per_queue"] = {q: sorted(v) for q, v in qstream.items()}
    beside = defaultdict(int)
    tot = 0
    kev_s = sorted(kev)
    for d in dsm:
        s0, e0 = d[0], d[1]
        tot += e0 - s0
        for s, e, n, q in kev_s:
            if s >= e0:
                break
            if e <= s0 or (s, e, n, q) == d:
                continue
            beside[n] += min(e, e0) - max(s, s0)
    out["beside_dsm_frac"] = {n: round(v / max(tot, 1), 3) for n, v in sorted(beside.items(), key=lambda kv: -kv[1])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
