"""The Python mirrors of the C-ABI structs (firedancer_amd/vtile.py, engine.py) against the C compiler's layout
of include/*.h: sizeof and every field's offset.  A field added on one side only would otherwise shift every
later field silently (the stats and config structs grow round by round)."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

from firedancer_amd import engine, vtile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PAIRS = [  # (C type, header, Python mirror)
    ("fdgpu_frag_meta_t", "fd_verify_gpu.h", vtile.FragMeta),
    ("fdgpu_vtile_done_t", "fd_verify_gpu.h", vtile.Done),
    ("fdgpu_vtile_gpu_metrics_t", "fd_verify_gpu.h", vtile.GpuMetrics),
    ("fdgpu_vtile_opts_t", "fd_verify_gpu.h", vtile.VTileOpts),
    ("fdgpu_stream_cfg_t", "fd_verify_gpu.h", vtile.StreamCfg),
    ("fdgpu_stream_stats_t", "fd_verify_gpu.h", vtile.StreamStats),
    ("fdgpu_debug_opts_t", "fd_ed25519_gpu.h", engine.DebugOpts),
]
DTYPES = [  # (C type, header, numpy dtype)
    ("fdgpu_txnm_t", "fd_verify_gpu.h", vtile.TXNM_DTYPE),
    ("fdgpu_txn_desc_t", "fd_ed25519_gpu.h", engine.DESC_DTYPE),
    ("fdgpu_txn_raw_t", "fd_ed25519_gpu.h", engine.RAW_DTYPE),
]
if hasattr(vtile, "TRACE_DTYPE"):
    DTYPES.append(("fdgpu_link_trace_t", "fd_verify_gpu.h", vtile.TRACE_DTYPE))
    DTYPES.append(("fdgpu_link_anomaly_t", "fd_verify_gpu.h", vtile.ANOM_DTYPE))


def _c_layout(items):
    """{ctype: (sizeof, {field: offset})} from gcc on the real headers."""
    lines = ["#include <stdio.h>", "#include <stddef.h>",
             f'#include "{ROOT}/include/fd_ed25519_gpu.h"', f'#include "{ROOT}/include/fd_verify_gpu.h"',
             "int main(void) {"]
    for ctype, fields in items:
        lines.append(f'  printf("%s size %zu\\n", "{ctype}", sizeof({ctype}));')
        for f in fields:
            lines.append(f'  printf("%s %s %zu\\n", "{ctype}", "{f}", offsetof({ctype}, {f}));')
    lines.append("  return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        r = subprocess.run(["gcc", "-std=gnu11", "-o", exe, src], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    lay = {}
    for ln in out.splitlines():
        t, f, v = ln.split()
        size, offs = lay.setdefault(t, [0, {}])
        if f == "size":
            lay[t][0] = int(v)
        else:
            offs[f] = int(v)
    return lay


def _public(names):
    return [n for n in names if not n.startswith("_")]


def test_ctypes_mirrors_match_c():
    items = [(c, _public([f for f, *_ in py._fields_])) for c, _, py in PAIRS]
    lay = _c_layout(items)
    for ctype, _, py in PAIRS:
        size, offs = lay[ctype]
        assert ctypes.sizeof(py) == size, (ctype, ctypes.sizeof(py), size)
        for f, *_ in py._fields_:
            if f in offs:
                assert getattr(py, f).offset == offs[f], (ctype, f, getattr(py, f).offset, offs[f])


@pytest.mark.parametrize("ctype,hdr,dt", DTYPES, ids=[d[0] for d in DTYPES])
def test_numpy_dtypes_match_c(ctype, hdr, dt):
    fields = _public(list(dt.names))
    lay = _c_layout([(ctype, fields)])
    size, offs = lay[ctype]
    assert dt.itemsize == size, (ctype, dt.itemsize, size)
    for f in fields:
        assert dt.fields[f][1] == offs[f], (ctype, f, dt.fields[f][1], offs[f])
