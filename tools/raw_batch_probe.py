#!/usr/bin/env python3
"""Latency of one async raw batch (the tile's batch shape) on one GPU: submit_raw of n 1232-byte
transactions, flush, blocking poll; p50/p99 over repeats, and the batch's GPU phases
(fdgpu_ed25519_phase_stats: launch -> kernels, kernels, end -> seen).  Run under rocprofv3 --kernel-trace
to see each kernel of the chain.  usage (GPU box): python tools/raw_batch_probe.py [n ...]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from firedancer_amd import Engine, synth
    from firedancer_amd.engine import load_library
    sizes = [int(x) for x in sys.argv[1:]] or [512, 1536, 4096]
    nmax = max(sizes)
    payload, desc, _, _ = synth.make_batch(nmax, synth.LARGE_NOOP, seed=9, threads=16)
    pays = [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    L = load_library()
    L.fdgpu_ed25519_phase_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulong)]
    for n in sizes:
        eng = Engine(device=0, max_txn=n, max_sig=n, max_payload=n * 1240 + 4096)
        eng.set_dedup(True, 7)
        lat = []
        for r in range(60):
            t0 = time.perf_counter()
            for i in range(n):
                assert eng.submit_raw(pays[i], i) == 0
            eng.flush()
            got = 0
            while got < n:
                tags, codes, fps, imgs, dtag = eng.poll_raw(n, True, dedup=True)[:5]
                got += len(codes)
                assert (codes == 0).all()
            if r >= 10:
                lat.append((time.perf_counter() - t0) * 1e3)
        ph = (ctypes.c_ulong * 9)()
        L.fdgpu_ed25519_phase_stats(eng.ctx, ph)
        nb = max(ph[0], 1)
        print(json.dumps({"n": n, "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                          "launch_to_kernels_us": ph[1] / nb * 1e-3, "kernels_us": ph[3] / nb * 1e-3,
                          "end_to_seen_us": ph[5] / nb * 1e-3}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
