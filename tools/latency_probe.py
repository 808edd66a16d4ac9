#!/usr/bin/env python3
"""Batch-latency breakdown on one GPU: for each batch size, the device-
resident verify (kernels only, HIP events) and the host-staged path
(pinned staging + H2D + kernels + D2H), p50/p99 over repeated calls.
usage (GPU box): python tools/latency_probe.py [sizes...]
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
    sizes = [int(x) for x in sys.argv[1:]] or [256, 1024, 4096, 8192, 16384, 65536]
    nmax = max(sizes)
    payload, desc, expect, nsig = synth.make_batch(nmax, synth.LARGE_NOOP, seed=7, threads=16)
    out = {}
    for n, path in [(n, p) for n in sizes for p in ("throughput", "latency8", "latency4", "latency2")]:
        lpay = payload[: int(desc["payload_off"][n - 1]) + 1232 + 64]
        d = desc[:n].copy()
        os.environ["FDGPU_DSM_LANES"] = path[-1] if path.startswith("latency") else "0"   # read at ctx creation
        eng = Engine(device=0, max_txn=n, max_sig=n, max_payload=lpay.nbytes)
        eng.set_small_batch_max(0 if path == "throughput" else 2**63)
        pay_d = torch.from_numpy(lpay).cuda()
        desc_d = torch.from_numpy(d.view(np.uint8)).cuda()
        o_d = torch.empty(n, dtype=torch.int8, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        dev, host = [], []
        for i in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, n, o_d.data_ptr(), None, st)
            torch.cuda.synchronize()
            if i >= 3:
                dev.append((time.perf_counter() - t0) * 1e3)
        eng.set_timing(True)
        eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, n, o_d.data_ptr(), None, st)
        torch.cuda.synchronize()
        kms = [eng.kernel_ms(k) for k in range(3)]
        eng.set_timing(False)
        assert (o_d.cpu().numpy() == 0).all()
        for i in range(30):
            t0 = time.perf_counter()
            lo, _ = eng.verify_txns_host(lpay, d, want_sig_codes=False)
            if i >= 3:
                host.append((time.perf_counter() - t0) * 1e3)
            assert (lo == 0).all()
        eng.close()
        out[(n, path)] = {"device_p50_ms": float(np.percentile(dev, 50)), "device_p99_ms": float(np.percentile(dev, 99)),
                  "host_p50_ms": float(np.percentile(host, 50)), "host_p99_ms": float(np.percentile(host, 99)),
                  "kernel_ms_prep_dsm_reduce": kms}
        print(n, path, json.dumps(out[(n, path)]), flush=True)


if __name__ == "__main__":
    main()
