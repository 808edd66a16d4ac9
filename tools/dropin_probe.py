#!/usr/bin/env python3
"""Latency of the link-level drop-in fd_ed25519_verify (one signature, one GPU round trip per call):
wall time per call (p50/p99 over N calls) -- run under rocprofv3 --kernel-trace to split it into kernels."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from firedancer_amd import engine, synth  # noqa: E402

payload, desc, _, _ = synth.make_batch(1, synth.LARGE_NOOP, seed=3)
d = desc[0]
raw = payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes()
sig = raw[d["signature_off"]: d["signature_off"] + 64]
pub = raw[d["acct_addr_off"]: d["acct_addr_off"] + 32]
msg = raw[d["message_off"]:]
assert engine.fd_ed25519_verify(msg, sig, pub) == 0
n = int(os.environ.get("N", 300))
ts = []
for _ in range(n):
    t0 = time.perf_counter()
    rc = engine.fd_ed25519_verify(msg, sig, pub)
    ts.append(time.perf_counter() - t0)
    assert rc == 0
ts = np.array(ts[20:]) * 1e6
print(json.dumps({"calls": len(ts), "p50_us": float(np.percentile(ts, 50)), "p99_us": float(np.percentile(ts, 99)),
                  "min_us": float(ts.min())}))
