#!/usr/bin/env python3
"""Run a sequence of configs[4] stream runs in ONE process (as bench.py does),
to see whether earlier runs affect later ones.
usage: tools/stream_seq.py tiles:rate:frags [tiles:rate:frags ...]   (env NPAY, BATCH, INFL, TORCH=1 to
allocate like bench.py first)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from firedancer_amd import synth, vtile  # noqa: E402

n_pay = int(os.environ.get("NPAY", 1 << 20))
payload, desc, _, _ = synth.make_batch(n_pay, synth.LARGE_NOOP, seed=77, threads=16)
if os.environ.get("TORCH") == "1":
    import torch
    keep = torch.from_numpy(payload).cuda()
for spec in sys.argv[1:]:
    tiles, rate, nf = spec.split(":")
    t0 = time.time()
    st = vtile.stream_bench(payload, desc["payload_off"], desc["payload_sz"], n_frags=int(float(nf)), tiles=int(tiles),
                            batch_txn=int(os.environ.get("BATCH", 8192)), max_inflight=int(os.environ.get("INFL", 1)),
                            mcache_depth=1 << 18, rate_fps=float(rate), zero_copy=True)
    print(json.dumps({"spec": spec, "wall": time.time() - t0, "fps": st["frags_per_s"], "p50": st["lat_p50_us"],
                      "p99": st["lat_p99_us"], "published": st["published"]}), flush=True)
