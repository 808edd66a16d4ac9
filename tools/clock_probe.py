#!/usr/bin/env python3
"""Shader clock during fd_dsm_kernel, measured: builds-free runner for the FD_CLOCK_PROBE engine
variant (build it first: tools/ab_build.sh clk -DFD_CLOCK_PROBE=1).  Runs the configs[1] batch
(1M single-signer 1232-byte txns, HBM-resident) a few times with per-kernel timing on and prints the
DSM's mean clock (s_memtime / s_memrealtime) and its duration."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FDGPU_LIB", os.path.join(ROOT, "build", "ab", "clk.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from firedancer_amd import Engine, load_library, synth  # noqa: E402

n = int(os.environ.get("TXNS", 1 << 20))
payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=1234, threads=16)
pay_d = torch.from_numpy(payload).cuda()
desc_d = torch.from_numpy(desc.view(np.uint8)).cuda()
out_d = torch.empty(n, dtype=torch.int8, device="cuda")
eng = Engine(device=0, max_txn=n, max_sig=nsig)
st = torch.cuda.current_stream().cuda_stream
L = load_library()
L.fdgpu_debug_dsm_clock_mhz.restype = ctypes.c_double
L.fdgpu_debug_dsm_clock_mhz.argtypes = [ctypes.c_ulong, ctypes.POINTER(ctypes.c_ulong)]
rows = []
for it in range(6):
    eng.set_timing(True)
    eng.verify_txns_device(pay_d.data_ptr(), desc_d.data_ptr(), n, nsig, out_d.data_ptr(), None, st)
    torch.cuda.synchronize()
    rec = ctypes.c_ulong()
    mhz = L.fdgpu_debug_dsm_clock_mhz((nsig + 255) // 256, ctypes.byref(rec))
    rows.append({"iter": it, "dsm_ms": eng.kernel_ms(1), "clock_mhz": mhz, "blocks": rec.value})
    eng.set_timing(False)
assert (out_d.cpu().numpy() == expect).all()
print(json.dumps({"dsm_clock": rows, "median_mhz": float(np.median([r["clock_mhz"] for r in rows[1:]]))}))
