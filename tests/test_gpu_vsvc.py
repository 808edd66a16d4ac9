"""GPU: several verify-tile processes on one GPU, served by one verify service (VERDICT r05 Missing 1).

The reference runs each verify tile as a process of its own, six by default (src/disco/topo/
fd_topo_run.c:66-153, src/app/fdctl/config/default.toml:788).  Here each served tile is the program
fdgpu_tile (a process of its own, no GPU context), and the process that owns the GPU is its verify service
(fdgpu_vsvc_*): the tiles hand it their frags through request rings, it batches the frags of all of them
together and returns every verdict to its tile.  The legs below run 2 and 3 tile processes on one GPU over
the configs[4] link (reliable; unreliable and lapped; paced on the latency path with the launch thread) and
compare every tile's verdicts, HA dedup tags and published records with the reference tile compiled in place
(oracle/_ref/libfdref_tile.so), exactly as tests/test_gpu_stream_parity.py does for tile threads.  They also
check that the tile processes never had the GPU open, that batches really mixed the tiles' frags, and the
service's fault path (a faulted engine context: its frags come back as FDGPU_VTILE_GPU_FAULT, later frags
verify on the recreated context).
"""
import ctypes
import itertools
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_stream_parity import payload_set, check_tiles, _with_hs_top  # noqa: E402

pytestmark = pytest.mark.gpu

N_FRAGS = 200_000
_seq = itertools.count()


def run_served(pays, reliable, depth, n_frags=N_FRAGS, tiles=2, zero_copy=True, **kw):
    from firedancer_amd import vtile
    sz = np.array([len(p) for p in pays], np.uint16)
    off = np.zeros(len(pays), np.uint32)
    off[1:] = np.cumsum(sz[:-1].astype(np.int64))
    arena = np.frombuffer(b"".join(pays) + bytes(64), np.uint8)
    cfg = dict(batch_txn=8192, max_inflight=2, rate_fps=0.0, nctx=1)
    cfg.update(kw)
    path = f"/dev/shm/fdgpu_tsvc_{os.getpid()}_{next(_seq)}"
    link = vtile.Link(path, create=True, payload=arena, off=off, sz=sz, n_frags=n_frags, tiles=tiles, gpus=1,
                      zero_copy=zero_copy, reliable=reliable, mcache_depth=depth, producers=1, svc=1, trace_cap=n_frags,
                      **cfg)
    try:
        assert link.run(0, 0, True) == 0
        st = link.result(timeout_s=120.0)
        traces = [link.trace(i, n_frags) for i in range(tiles)]
        svc = link.svc_stats()
    finally:
        link.close()
        if os.path.exists(path):
            os.unlink(path)
    return st, traces, svc


def test_numa_node_sysfs_matches_bus_id():
    """The host plan's and the served link's GPU -> NUMA node (sysfs alone, no GPU call) is the HIP device's
    own (its PCI bus id)."""
    from firedancer_amd import engine, vtile
    L = engine.load_library()
    for d in range(int(os.environ.get("FDGPU_TEST_DEVICES", "1"))):
        assert vtile.gpu_numa_node(d) == int(L.fdgpu_device_numa_node(d))


@pytest.mark.parametrize("tiles", [2, 3])
def test_served_parity_reliable(tiles):
    pays = payload_set()
    st, traces, svc = run_served(pays, reliable=True, depth=1 << 16, tiles=tiles)
    assert st["verdicts"] == N_FRAGS and st["lost"] == 0 and st["overruns"] == 0
    assert st["tiles_gpu_open"] == 0, "a served tile process had the GPU open"
    assert svc["completed"] == N_FRAGS and svc["fault_completions"] == 0
    assert svc["mixed_batches"] > 0, "no batch held the frags of more than one tile"
    seen = list(check_tiles(pays, traces, tiles=tiles))
    assert sum(k for _, k, _ in seen) == N_FRAGS
    assert all(m[2] > 0 and m[1] > 0 for _, _, m in seen), "the stream should exercise dedup and verify failures"


def test_served_parity_host_copy():
    """The reference's own intake (during_frag copies the frag into the tile's out dcache, fd_verify_tile.c:79):
    the service's GPU batch reads each record from its tile's out dcache in the service's segment."""
    pays = payload_set()
    st, traces, svc = run_served(pays, reliable=True, depth=1 << 16, tiles=2, zero_copy=False)
    assert st["verdicts"] == N_FRAGS and st["lost"] == 0 and st["tiles_gpu_open"] == 0
    assert svc["completed"] == N_FRAGS and svc["mixed_batches"] > 0
    seen = list(check_tiles(pays, traces, tiles=2))
    assert sum(k for _, k, _ in seen) == N_FRAGS


def test_served_parity_unreliable_laps():
    pays = payload_set()
    st, traces, svc = run_served(pays, reliable=False, depth=1 << 12, tiles=2)
    assert st["verdicts"] + st["lost"] == N_FRAGS and st["lost"] > 0
    n_ovr = sum(int((t["result"] == 5).sum()) for t in traces)      # FDGPU_VTILE_OVERRUN
    assert n_ovr == st["overruns"]
    seen = list(check_tiles(pays, traces, tiles=2))
    assert sum(k for _, k, _ in seen) == st["verdicts"] - st["overruns"]


@pytest.mark.parametrize("tiles", [3])
def test_served_parity_paced_latency(tiles):
    """The bench's paced configuration served: three tile processes, the service with two staggered engine
    contexts on the latency path, exclusive CUs, 16 CUs for the copies, copies after 25 us, the launch
    thread -- at 7.5M frags/s on the device.  Nothing lost or overrun; frag for frag the reference's."""
    n = 250_000
    pays = _with_hs_top(payload_set())
    st, traces, svc = run_served(pays, reliable=False, depth=1 << 18, n_frags=n, tiles=tiles, rate_fps=7.5e6, nctx=2,
                                 max_inflight=1, gather_cus=16, copy_wait_ns=25_000, launcher=1)
    assert st["lost"] == 0 and st["overruns"] == 0 and st["verdicts"] == n, (st["lost"], st["overruns"])
    assert st["batches"] > 0 and st["batch_txns"] / st["batches"] <= 8192
    assert svc["gm"]["launcher"][0] >= st["batches"]
    seen = list(check_tiles(pays, traces, tiles=tiles))
    assert sum(k for _, k, _ in seen) == n


class _InProc:
    """A service and one served tile in this process (the service's loop driven by hand), over an in link
    of host memory the service maps as its regions 0 (records) and 1 (mcache lines)."""

    def __init__(self, n_rec=1024, depth=4096, debug_hooks=1):
        from firedancer_amd import vtile
        self.vt = vtile
        L = vtile.load()
        self.L = L
        self.svc = vtile.Service(None, create=True, clients=1, batch_txn=1024, nctx=2, max_inflight=1,
                                  debug_hooks=debug_hooks)
        self.mc = L.fdgpu_mcache_new(depth, 0)
        self.lines = L.fdgpu_mcache_lines(self.mc)
        self.buf = np.zeros(n_rec * 24 * 64 + 8192, np.uint8)
        self.base = (self.buf.ctypes.data + 4095) & ~4095
        self.rsz = n_rec * 24 * 64
        assert self.svc.add_region(0, self.base, self.rsz) == 0
        assert self.svc.add_region(1, self.lines, depth * 32) == 0
        self.tile = vtile.VTile(service=self.svc, client=0, seed=0x1234)
        assert self.tile.set_svc_region(0, self.base, self.rsz) == 0
        assert self.tile.set_svc_region(1, self.lines, depth * 32) == 0
        assert self.tile.set_in_links([self.mc]) == 0
        assert self.svc.start(0) == 0
        self.chunk, self.seq = 0, 0

    def feed(self, payloads):
        for p in payloads:
            rec = self.vt.frag_bytes(p)
            c = self.chunk
            self.chunk = (self.chunk + (len(rec) + 127) // 128 * 2) % (self.rsz // 64 - 48)
            o = self.base - self.buf.ctypes.data + c * 64
            self.buf[o:o + len(rec)] = np.frombuffer(rec, np.uint8)
            self.L.fdgpu_mcache_publish(self.mc, self.seq, 0, c, len(rec), 0, 0)
            assert self.tile.during_frag_at(self.base + c * 64, len(rec), self.seq) == 0
            self.seq += 1

    def drain(self, n, faults_at=None):
        out = []
        self.tile.housekeep()
        for i in range(200000):
            if faults_at is not None and i == faults_at:
                self.tile.debug_fault(0)
                self.tile.debug_fault(1)
            self.svc.poll()
            self.tile.housekeep()
            if i % 8 == 7:
                self.tile.flush()
            out += self.tile.after_frags(4096)
            if len(out) >= n:
                return out
        raise AssertionError(f"only {len(out)} of {n} verdicts")


def test_served_in_process_codes_and_fault_recovery():
    from firedancer_amd import synth
    payload, desc, expect, _ = synth.make_batch(600, synth.LARGE_NOOP, invalid_frac=0.25, seed=7)
    pays = [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    want = [0 if e == 0 else 2 for e in expect]          # FDGPU_VTILE_PUBLISH / _VERIFY_FAIL
    r = _InProc()
    try:
        _in_process_phases(r, pays, want)
    finally:                                             # (before the interpreter's exit tears HIP down)
        r.tile.close(); r.svc.close()


def test_served_tile_cannot_fault_the_service_without_debug_hooks():
    """fdgpu_vtile_debug_fault is a test hook: a service made without cfg.debug_hooks ignores a tile's request
    to fault its engine contexts, and every frag verifies."""
    from firedancer_amd import synth
    payload, desc, expect, _ = synth.make_batch(200, synth.LARGE_NOOP, invalid_frac=0.25, seed=8)
    pays = [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    want = [0 if e == 0 else 2 for e in expect]
    r = _InProc(debug_hooks=0)
    try:
        r.feed(pays)
        out = r.drain(200, faults_at=0)
        assert [d[0] for d in out] == list(range(200)) and [d[1] for d in out] == want
        st = r.svc.stats()
        assert st["faults"] == 0 and st["fault_completions"] == 0
    finally:
        r.tile.close(); r.svc.close()


def _in_process_phases(r, pays, want):
    r.feed(pays[:200])
    out = r.drain(200)
    assert [d[0] for d in out] == list(range(200)) and [d[1] for d in out] == want[:200]
    # both engine contexts faulted while frags are pending: those come back as GPU_FAULT, in order
    r.feed(pays[200:400])
    out = r.drain(200, faults_at=0)
    assert [d[0] for d in out] == list(range(200, 400))
    res = [d[1] for d in out]
    assert res.count(6) > 0                               # FDGPU_VTILE_GPU_FAULT
    assert all(x == 6 or x == w for x, w in zip(res, want[200:400]))
    # the service recreated its contexts: later frags verify again
    r.feed(pays[400:600])
    out = r.drain(200)
    assert [d[1] for d in out] == want[400:600]
    st = r.svc.stats()
    assert st["recovered"] >= 1 and st["fault_completions"] == res.count(6)


def test_launch_thread_failure_does_not_hang_blocking_drain():
    """a batch launch that fails on the tile's launch thread faults the context asynchronously;
    a blocking after_frags then returns that context's frags as GPU_FAULT instead of waiting forever."""
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(64, synth.LARGE_NOOP, seed=9)
    pays = [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    t = vtile.VTile(device=0, batch_txn=256, nctx=1, launcher=1)
    try:
        t.debug_fail_launch(0)
        for s, p in enumerate(pays):
            assert t.during_frag(vtile.frag_bytes(p), s) == 0
        out = t.after_frags(256, blocking=True)           # (pytest's timeout ends a hang)
        assert [d[0] for d in out] == list(range(64)) and all(d[1] == vtile.GPU_FAULT for d in out)
        assert t.faulted() == 1
    finally:
        t.close()


@pytest.mark.parametrize("zero_copy", [False, True])
def test_served_vtile_vs_reference_tile(oracle, zero_copy):
    """A served tile over the mixed stream of tests/test_gpu_vtile.py -- valid / invalid signatures, parse
    failures, HA duplicates (with tcache eviction) and bundles with failing members -- with the service driven
    by hand in this process: per-frag outcomes, metrics, published records and dedup tags are the reference
    tile's (fd_verify_tile.c:103-157), on the host-copy intake and on the zero-copy one."""
    pytest.importorskip("xxhash")
    from test_gpu_vtile import make_stream, expectation, in_dcache
    from firedancer_amd import vtile
    frags = make_stream(seed=13)
    seed, depth = 0x77aa55, 1 << 12
    want_res, want_m, want_recs, want_tags = expectation(oracle, frags, seed, depth)
    L = vtile.load()
    svc = vtile.Service(None, create=True, clients=1, batch_txn=256, nctx=2, max_inflight=1)
    fbs = [vtile.frag_bytes(p, b) for p, b in frags]
    buf, offs = in_dcache(fbs)
    mdepth = 1 << 12
    mc = L.fdgpu_mcache_new(mdepth, 0)
    lines = L.fdgpu_mcache_lines(mc)
    lo = buf.ctypes.data & ~4095
    rsz = ((buf.ctypes.data + buf.size + 4095) & ~4095) - lo
    t = None
    try:
        assert svc.add_region(0, lo, rsz) == 0 and svc.add_region(1, lines, mdepth * 32) == 0
        t = vtile.VTile(service=svc, client=0, tcache_depth=depth, seed=seed)
        assert t.set_svc_region(0, lo, rsz) == 0 and t.set_svc_region(1, lines, mdepth * 32) == 0
        if zero_copy:
            assert t.set_in_links([mc]) == 0
        assert svc.start(0) == 0
        got, bad = [], []

        def drain(n_want):
            for _ in range(200000):
                svc.poll()
                t.housekeep()
                for seq, r, chunk, sz, tag, _ in t.after_frags(4096):
                    got.append((seq, r))
                    if r == vtile.PUBLISH:
                        head, timg = want_recs.get(seq, (b"", b""))
                        rec = t.record(chunk, sz)
                        if rec[: len(head)] != head or rec[(len(head) + 1) & ~1:] != timg:
                            bad.append(seq)
                        if want_tags is not None and tag != want_tags.get(seq):
                            bad.append(("tag", seq))
                if len(got) >= n_want:
                    return
                t.flush()
            raise AssertionError(f"{len(got)} of {n_want} verdicts")

        for seq, fb in enumerate(fbs):
            if zero_copy:
                L.fdgpu_mcache_publish(mc, seq, 0, (buf.ctypes.data + offs[seq] - lo) // 64, len(fb), 0, 0)
                rc = t.during_frag_at(buf.ctypes.data + offs[seq], len(fb), seq)
            else:
                rc = t.during_frag(fb, seq)
            assert rc == 0, (seq, rc)
            if seq % 97 == 96:
                drain(seq + 1 - 32)
        drain(len(frags))
        assert [g[0] for g in got] == list(range(len(frags)))
        assert [g[1] for g in got] == want_res
        assert t.metrics() == want_m
        assert bad == []
        assert sum(want_m[:4]) > 100 and want_m[2] > 10 and want_m[3] > 0
    finally:
        if t is not None:
            t.close()
        svc.close()


_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
from firedancer_amd import vtile
link = vtile.Link(sys.argv[2], create=False, timeout_s=120.0)
try:
    rc = link.run(1, 0, True)          # process 1: its service (device 0 here) and its tiles 1, 3
finally:
    link.close()
sys.exit(0 if rc == 0 else 3)
"""


def test_served_two_processes_parity(engine_path):
    """The N = 2 wiring of the served stream with both processes on this one GPU: process 0 creates the link and
    runs the producer, and each process runs the verify service of "its GPU" with its tile processes (tile i ->
    process i % 2, fd_verify_tile.c:47-48).  Every tile's verdicts, tags and records against the reference tile."""
    import subprocess
    from firedancer_amd import engine, vtile
    if engine_path != "throughput":
        pytest.skip("the child process runs the product's defaults: runs once, on them")
    engine.debug_reset_opts()
    pays = payload_set()
    sz = np.array([len(p) for p in pays], np.uint16)
    off = np.zeros(len(pays), np.uint32)
    off[1:] = np.cumsum(sz[:-1].astype(np.int64))
    arena = np.frombuffer(b"".join(pays) + bytes(64), np.uint8)
    n = 100_000
    path = f"/dev/shm/fdgpu_tsvc2_{os.getpid()}"
    link = vtile.Link(path, create=True, payload=arena, off=off, sz=sz, n_frags=n, tiles=4, gpus=2, zero_copy=True,
                      reliable=True, mcache_depth=1 << 16, producers=1, svc=1, trace_cap=n, batch_txn=8192,
                      max_inflight=2, rate_fps=0.0, nctx=1)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = subprocess.Popen([sys.executable, "-c", _CHILD, root, path])
    try:
        assert link.run(0, 0, True) == 0
        assert child.wait(timeout=180) == 0
        st = link.result(timeout_s=60.0)
        traces = [link.trace(i, n) for i in range(4)]
    finally:
        if child.poll() is None:
            child.kill()
        link.close()
        if os.path.exists(path):
            os.unlink(path)
    assert st["verdicts"] == n and st["lost"] == 0 and st["tiles_gpu_open"] == 0
    seen = list(check_tiles(pays, traces, tiles=4))
    assert sum(k for _, k, _ in seen) == n
