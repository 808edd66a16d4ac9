#!/usr/bin/env python3
"""Sweep the configs[4] streaming harness (fdgpu_stream_bench) over tile
count / batch size on one GPU; prints one JSON line per point."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from firedancer_amd import synth, vtile  # noqa: E402

n_pay = int(os.environ.get("NPAY", 1 << 18))
t = time.time()
payload, desc, _, _ = synth.make_batch(n_pay, synth.LARGE_NOOP, seed=77, threads=16)
print(json.dumps({"gen_s": time.time() - t}), flush=True)
for tiles in [int(x) for x in os.environ.get("TILES", "1,2,4,8").split(",")]:
    for batch in [int(x) for x in os.environ.get("BATCH", "1024,4096").split(",")]:
        for rate in [float(x) for x in os.environ.get("RATE", "0").split(",")]:
          for infl in [int(x) for x in os.environ.get("INFL", "2").split(",")]:
           for nf in [int(x) for x in os.environ.get("NF", "1000000").split(",")]:
            for zc in [int(x) for x in os.environ.get("ZC", "0").split(",")]:
             st = vtile.stream_bench(payload, desc["payload_off"], desc["payload_sz"], n_frags=nf,
                                     tiles=tiles, batch_txn=batch, max_inflight=infl,
                                     mcache_depth=int(os.environ.get("DEPTH", 1 << 16)), rate_fps=rate, zero_copy=bool(zc))
             st.update(tiles=tiles, batch=batch, rate=rate, inflight=infl, zero_copy=zc)
             print(json.dumps(st), flush=True)
