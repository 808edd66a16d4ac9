#!/usr/bin/env python3
"""Debug the half-size path on the configs[3] batch: which signatures differ from the oracle, by
launch position, under host (pipelined) and device (one launch) paths and forced-slow settings."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import torch
    import firedancer_amd as fa
    from firedancer_amd import synth
    from oracle.oracle import Oracle
    n = int(os.environ.get("NTX", 1 << 18))
    payload, desc, expect, nsig = synth.make_batch(n, synth.MULTI, 12, 0.1, seed=777, threads=16)
    eng = fa.Engine(device=0, max_txn=n, max_sig=nsig, max_payload=payload.nbytes)
    mode = os.environ.get("MODE", "host")
    if mode == "host":
        t, s = eng.verify_txns_host(payload, desc)
    else:
        pd = torch.from_numpy(payload).cuda(); dd = torch.from_numpy(desc.view(np.uint8)).cuda()
        to = torch.empty(n, dtype=torch.int8, device="cuda"); so = torch.empty(nsig, dtype=torch.int8, device="cuda")
        eng.verify_txns_device(pd.data_ptr(), dd.data_ptr(), n, nsig, to.data_ptr(), so.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize(); t, s = to.cpu().numpy(), so.cpu().numpy()
    bad_t = np.nonzero(t != expect)[0]
    o_t, o_s = Oracle().verify_txns(payload, desc, nsig, threads=16) if len(bad_t) else (None, None)
    out = {"mode": mode, "env": {k: os.environ.get(k) for k in ("FDGPU_HALF", "FDGPU_HALF_FORCE_SLOW", "NTX")},
           "nsig": int(nsig), "bad_txn": int(len(bad_t))}
    if len(bad_t):
        bad_s = np.nonzero(s != o_s)[0]
        out.update(bad_sig=int(len(bad_s)), first_bad_sig=bad_s[:10].tolist(), last_bad_sig=bad_s[-5:].tolist(),
                   got=s[bad_s[:10]].tolist(), want=o_s[bad_s[:10]].tolist(),
                   hist=np.histogram(bad_s, bins=8, range=(0, nsig))[0].tolist())
    print(json.dumps(out))
    sys.exit(0)

for v in sys.argv[1:]:
    env = dict(os.environ)
    for kv in filter(None, v.split(";")):
        k, val = kv.split("="); env[k] = val
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True, text=True,
                       timeout=300)
    print(v, "->", r.stdout.strip().splitlines()[-1] if r.stdout.strip() else f"rc {r.returncode} {r.stderr[-800:]}",
          flush=True)
