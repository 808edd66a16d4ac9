#!/usr/bin/env python3
"""Tabulate the configs[4] stream legs of bench detail files (one per A/B arm): max-rate sigs/s, the tile
host split, gather stats, paced p50/p99 per rate.  usage: ab_stream_table.py DIR [DIR ...] (reads *.json)"""
import glob
import json
import os
import sys

for d in sys.argv[1:]:
    for p in sorted(glob.glob(os.path.join(d, "*.json"))):
        try:
            rec = json.load(open(p))
        except (OSError, ValueError):
            continue
        s = rec.get("stream")
        if not isinstance(s, dict) or "max_rate" not in s:
            continue
        mx, ur = s["max_rate"], s.get("unreliable_max") or {}
        g = mx.get("gather_gpu") or {}
        curve = " ".join(f"{r/1e6:g}M:{p50/1e3:.2f}/{p99/1e3:.2f}" for r, p50, p99 in
                         ((c["rate_fps"], c["p50_us"], c["p99_us"]) for c in s.get("latency_curve") or []))
        print(f"{os.path.basename(p)[:-5]:10s} head {rec['value']/1e6:6.1f}M  max {mx['sigs_per_s']/1e6:5.2f}M "
              f"host {mx.get('tile_host_ns_per_frag')} batch {mx.get('mean_batch_txns', 0):7.0f} "
              f"gather {g.get('run_mean_us', 0):5.1f}us l2s {g.get('launch_to_start_mean_us', 0):6.0f}us "
              f"refus {mx.get('copy_backlog_refusals', 0)/1e6:5.1f}M huge {mx.get('anon_huge_mb')} "
              f"unrel {ur.get('sigs_per_s', 0)/1e6:5.2f}M cpu {(mx.get('host_cpu') or {}).get('tile_share_min')} "
              f"ivcsw {(mx.get('host_cpu') or {}).get('tile_nivcsw')} | {curve}")
