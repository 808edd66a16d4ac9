#!/usr/bin/env python3
"""Soak the engine on the GPU: many seeds of the BASELINE mixes, each verified several times.

configs[2] (1M txns, 10 % adversarial) and configs[3] (256K txns, 1-12 signers, 10 % invalid) go
through the throughput path (verify_txns_device). Slices of 8192 txns of the configs[3] batch go
through the host-staged latency path (verify_txns_host). Every run is compared with the generator's
intended codes, which the GPU parity tests pin against the oracle and the reference. Repeated runs of
one input must also agree with each other; a race such as the slow-list one in DESIGN.md §3b shows up
as a mismatch. One JSON line per seed, then a summary line.

usage: python tools/soak.py [seeds] [repeats]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import synth  # noqa: E402
from firedancer_amd.engine import Engine  # noqa: E402

seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
threads = min(16, os.cpu_count() or 1)
bad, total_sigs = 0, 0
t0 = time.time()
mixes = (("configs2", synth.LARGE_NOOP, 1 << 20, 1, 0.1), ("configs3", synth.MULTI, 1 << 18, 12, 0.1))
engines = {name: Engine(device=0, max_txn=nt, max_sig=nt * ms) for name, _, nt, ms, _ in mixes}
leng = Engine(device=0, max_txn=8192, max_sig=8192 * 12, max_payload=8192 * 1232 + 4096)
for s in range(seeds):
    rec = {"seed": s}
    for name, kind, nt, ms, inv in mixes:
        pay, desc, expect, nsig = synth.make_batch(nt, kind, ms, inv, seed=9000 + s, threads=threads)
        dp = torch.from_numpy(pay).cuda()
        dd = torch.from_numpy(desc.view(np.uint8)).cuda()
        out = torch.empty(nt, dtype=torch.int8, device="cuda")
        first, mism = None, 0
        for _ in range(reps):
            engines[name].verify_txns_device(dp.data_ptr(), dd.data_ptr(), nt, nsig, out.data_ptr(), None, None)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            mism += int(np.count_nonzero(got != expect))
            if first is None:
                first = got
            elif not np.array_equal(first, got):
                mism += 1
            total_sigs += nsig
        rec[name] = {"sigs": nsig, "mismatches": mism,
                     "slow_listed": int(engines[name].L.fdgpu_ed25519_slow_count(engines[name].ctx))}
        bad += mism
        if name == "configs3":            # latency path: host-staged 8192-txn slices of the same batch
            lm = 0
            for off in range(0, nt, 8192 * 8):
                sl = slice(off, off + 8192)
                base = int(desc["payload_off"][off])
                end = int(desc["payload_off"][off + 8191]) + int(desc["payload_sz"][off + 8191])
                ld = desc[sl].copy()
                ld["payload_off"] -= base
                ld["sig_base"] -= ld["sig_base"][0]
                for _ in range(reps):
                    got, _sc = leng.verify_txns_host(pay[base:end + 64], ld, want_sig_codes=False)
                    lm += int(np.count_nonzero(got != expect[sl]))
                    total_sigs += int(ld["sig_cnt"].astype(np.int64).sum())
            rec["latency_slices"] = {"mismatches": lm}
            bad += lm
        del dp, dd, out
    rec["elapsed_s"] = round(time.time() - t0, 1)
    print(json.dumps(rec), flush=True)
print(json.dumps({"soak": "done", "seeds": seeds, "repeats": reps, "sigs_verified": total_sigs,
                  "mismatches": bad, "ok": bad == 0}), flush=True)
sys.exit(1 if bad else 0)
