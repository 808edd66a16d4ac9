#!/usr/bin/env python3
"""One line per stream leg of each A/B result file of tools/gpu_stream_ab.sh (bench.py --stream-child output)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads([x for x in open(f).read().splitlines() if x.startswith("{")][-1])
    print(f"== {f}")
    for leg, v in d["legs"].items():
        g = v.get("gather_gpu", {})
        print(f"  {leg:14s} sigs/s {v['sigs_per_s']/1e6:6.2f}M verdicts {v['verdicts']:>10d} lost {v['lost']:>9d} "
              f"ovr {v['overruns_at_verdict']:>8d} pub {v['published']:>10d} p50 {v['p50_us']/1e3:7.2f} "
              f"p99 {v['p99_us']/1e3:7.2f} max {v['max_us']/1e3:7.2f} ms | host {v['tile_host_ns_per_frag']} "
              f"wait {v['tile_after_split_ns_per_frag']['gpu_wait_ns']} | copy lat {v['copy_lat_mean_us']:.0f}/"
              f"{v['copy_lat_max_us']:.0f} us, gather start {g.get('launch_to_start_mean_us', 0):.0f}/"
              f"{g.get('launch_to_start_max_us', 0):.0f} us, batch {v['mean_batch_txns']:.0f}")
        if v.get("tile_prof_ns_per_frag"):
            print("      prof ns/frag: " + ", ".join(f"{k} {x}" for k, x in v["tile_prof_ns_per_frag"].items()))
        ph = v.get("batch_phases_us")
        if ph:
            print("      phases us: " + ", ".join(f"{k} {x:.0f}" for k, x in ph.items() if x is not None))
