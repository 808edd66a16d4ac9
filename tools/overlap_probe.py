#!/usr/bin/env python3
"""Throughput of back-to-back 1M-signature device batches: one context on
one stream vs two contexts on two streams, alternating batches (the next
batch's prep can fill the SIMDs a batch's DSM tail leaves idle).
usage (GPU box): python tools/overlap_probe.py [steps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from firedancer_amd import Engine, synth
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = 1 << 20
    payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=5, threads=16)
    pay_d = torch.from_numpy(payload).cuda()
    desc_d = torch.from_numpy(desc.view(np.uint8)).cuda()
    for nstream in (1, 2, 1, 2):
        engs = [Engine(device=0, max_txn=n, max_sig=nsig) for _ in range(nstream)]
        strs = [torch.cuda.Stream() for _ in range(nstream)]
        outs = [torch.empty(n, dtype=torch.int8, device="cuda") for _ in range(nstream)]

        def step(i):
            k = i % nstream
            engs[k].verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, outs[k].data_ptr(), None,
                                       strs[k].cuda_stream)
        for i in range(2 * nstream):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = all(bool(np.array_equal(o.cpu().numpy(), expect)) for o in outs)
        print(json.dumps({"streams": nstream, "sigs_per_s": nsig * steps / dt, "ms_per_step": dt * 1e3 / steps,
                          "ok": ok}), flush=True)
        for e in engs:
            e.close()


if __name__ == "__main__":
    main()
