#!/usr/bin/env python3
"""Sweep the configs[4] verify stage on one GPU (fdgpu_stream_run: one producer link, T verify tiles,
tile i -> GPU 0): one JSON line per point.  Env: TILES, RATE (frags/s, 0 = max), REL (1 reliable /
0 unreliable), SECONDS, BATCH, INFL, ZC, DEPTH (mcache lines), PROD (producer links), VARIANTS (comma list of env assignments applied per point,
e.g. "FDGPU_VTILE_GPU_TAG=1,FDGPU_VTILE_GPU_TAG=0"), NPAY (distinct payloads)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import synth, vtile  # noqa: E402


def lat_q(hist, q):
    tot = sum(hist)
    c = 0
    for i, h in enumerate(hist):
        c += h
        if tot and c > q * tot:
            return 32 * 2 ** (i / 4)            # bucket upper edge, us
    return None


n_pay = int(os.environ.get("NPAY", 1 << 20))
t = time.time()
payload, desc, _, _ = synth.make_batch(n_pay, synth.LARGE_NOOP, seed=77, threads=16)
print(json.dumps({"gen_s": time.time() - t}), flush=True)
secs = float(os.environ.get("SECONDS", 5))
variants = [v for v in os.environ.get("VARIANTS", "").split(",") if v] or [""]
for var in variants:
    if var:
        k, v = var.split("=")
        os.environ[k] = v
    for rel in [int(x) for x in os.environ.get("REL", "1,0").split(",")]:
        for tiles in [int(x) for x in os.environ.get("TILES", "2,6").split(",")]:
            for rate in [float(x) for x in os.environ.get("RATE", "0,2e6").split(",")]:
                nf = int((rate or 8e6) * secs)
                st = vtile.stream_run(payload, desc["payload_off"], desc["payload_sz"], n_frags=nf, tiles=tiles,
                                      batch_txn=int(os.environ.get("BATCH", 8192)),
                                      max_inflight=int(os.environ.get("INFL", 1)), mcache_depth=int(os.environ.get("DEPTH", 1 << 18)),
                                      rate_fps=rate, zero_copy=bool(int(os.environ.get("ZC", 1))), reliable=bool(rel),
                                      producers=int(os.environ.get("PROD", 1)))
                n = max(st["verdicts"], 1)
                print(json.dumps({"variant": var, "reliable": rel, "tiles": tiles, "rate": rate, "frags": st["frags"],
                                  "verdicts": st["verdicts"], "lost": st["lost"], "overruns": st["overruns"],
                                  "sigs_per_s": round(st["sigs_per_s"]), "p50_us": st["lat_p50_us"],
                                  "p99_us": st["lat_p99_us"], "max_us": st["lat_max_us"],
                                  "host_ns": [round(x / n, 1) for x in st["tile_ns"]], "wait_poll_after_ns": [round(st[k] / n, 1) for k in ("gpu_wait_ns", "poll_ns", "after_ns", "launch_ns")], "idle_ns": round(st["tile_idle_ns"] / n, 1),
                                  "prod_s": round(st["prod_seconds"], 3), "prod_wait_s": round(st["prod_wait_ns"] * 1e-9, 3),
                                  "seconds": round(st["seconds"], 3), "prof_ns": [round(x / n, 1) for x in st["prof_ns"]],
                                  "batches": st["batches"], "mean_batch": round(st["batch_txns"] / max(st["batches"], 1)),
                                  "inflight_max": st["inflight_max"], "gpu_lat_p50_us": lat_q(st["gpu_lat_hist"], .5),
                                  "gpu_lat_p99_us": lat_q(st["gpu_lat_hist"], .99), "metrics": st["metrics"]}),
                      flush=True)
