#!/usr/bin/env python3
"""Length of each role of the latency path's prep, measured: runner for the FD_PREP_PROBE engine variant
(build it first: tools/ab_build.sh pp -DFD_PREP_PROBE=1).  Runs HBM-resident batches of TXNS (default
2,800, the paced leg's mean batch at 10M frags/s) single-signer 1232-byte transactions through the
latency path and prints, per role of fd_prep_kernel (0 decode A + -A table, 1 decode R + -R table,
2 S check + SHA-512 + half-size reduction), the mean and max wave duration and the role's span from
the kernel's first wave start, in microseconds (100 MHz real-time counter)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FDGPU_LIB", os.path.join(ROOT, "build", "ab", "pp.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from firedancer_amd import Engine, load_library, synth  # noqa: E402

n = int(os.environ.get("TXNS", 2800))
if os.environ.get("QUAD_SHA"):                # -1: the hash role on one lane per signature (fdgpu_debug_opts_t.quad_sha)
    from firedancer_amd import engine as _engine
    _engine.debug_set_opts(quad_sha=int(os.environ["QUAD_SHA"]))
reps = int(os.environ.get("REPS", 20))
payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=1234, threads=8)
pay_d = torch.from_numpy(payload).cuda()
desc_d = torch.from_numpy(desc.view(np.uint8)).cuda()
out_d = torch.empty(n, dtype=torch.int8, device="cuda")
eng = Engine(device=0, max_txn=n, max_sig=nsig)
st = torch.cuda.current_stream().cuda_stream
L = load_library()
probe = hasattr(L, "fdgpu_debug_prep_probe")     # the plain library: just the batches (for a kernel trace)
if probe:
    L.fdgpu_debug_prep_probe.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
nw = min(6 * ((nsig + 255) // 256) * 4, 4096)     # waves of the launch (6 sg blocks with the quad hash role)
rows = []
for it in range(reps):
    if probe:
        L.fdgpu_debug_prep_probe_clear()
    eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, out_d.data_ptr(), None, st)
    torch.cuda.synchronize()
    if not probe:
        continue
    buf = np.zeros((nw, 3), np.uint64)
    assert L.fdgpu_debug_prep_probe(buf.ctypes.data, nw) == 0
    buf = buf[buf[:, 1] > 0].astype(np.int64)
    t0 = buf[:, 0].min()
    r = {}
    for role in range(3):
        b = buf[buf[:, 2] == role]
        if not len(b):
            continue
        d = (b[:, 1] - b[:, 0]) / 100.0
        r[role] = {"waves": int(len(b)), "mean_us": float(d.mean()), "max_us": float(d.max()),
                   "span_us": float((b[:, 1].max() - t0) / 100.0), "start_spread_us": float((b[:, 0].max() - t0) / 100.0)}
    rows.append(r)
if not os.environ.get("PROBE_NOCHECK"):       # FD_PREP_PROBE=2 / 3 builds stop the hash role early (wrong codes)
    assert (out_d.cpu().numpy() == expect).all()
summ = {}
for role in range(3):
    v = [r[role] for r in rows[2:] if role in r]
    if v:
        summ[role] = {k: float(np.median([x[k] for x in v])) for k in ("waves", "mean_us", "max_us", "span_us", "start_spread_us")}
print(json.dumps({"txns": n, "sigs": int(nsig), "reps": reps, "median_over_reps": summ}))
