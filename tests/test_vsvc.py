"""The verify service's rings and a served tile, on the CPU (no GPU call anywhere in this file).

A served verify tile (fdgpu_vtile_new_svc) hands each frag to its GPU's verify service through a request
ring and drains verdicts from a completion ring (include/fd_verify_gpu.h, fdgpu_vsvc_*).  Here the
service's GPU side is the CPU loopback fdgpu_vsvc_debug_serve: it completes each request with a code the
test picks, copies the record into the tile's out dcache, makes the overrun check and computes the HA
dedup tag with the tile's seed.  What is checked is the served tile's half: request contents and order,
completions back in frag order, after_frag's decisions on them (publish / verify fail / parse fail / dedup /
overrun / GPU fault, fd_verify_tile.c:103-157), the copied prefix that a reliable link's credit waits for,
and the fault path when the service stops beating.  The GPU service itself, against the reference tile, is
tests/test_gpu_vsvc.py.
"""
import ctypes
import os
import time

import numpy as np
import pytest

from firedancer_amd import vtile

CHUNK = vtile.CHUNK_SZ
FP = 100                       # the loopback's fd_txn_t footprint


def _payload(i: int, sz: int = 200) -> bytes:
    rng = np.random.default_rng(i)
    b = bytearray(rng.integers(0, 256, sz, dtype=np.uint8).tobytes())
    b[0] = 1                   # one signature, at bytes 1..64
    return bytes(b)


class Rig:
    """One service segment with `clients` served tiles reading one in link (an mcache + an in dcache in host
    memory, both regions of the service)."""

    def __init__(self, clients=1, depth=1024, n_rec=256, seeds=None, zero_copy=True, **opts):
        self.svc = vtile.Service(None, create=True, clients=clients, batch_txn=1024)
        L = vtile.load()
        self.L = L
        self.depth = depth
        self.mc = L.fdgpu_mcache_new(depth, 0)
        self.lines = L.fdgpu_mcache_lines(self.mc)
        self.in_dc = np.zeros(n_rec * 32 * CHUNK + 4096, np.uint8)
        base = self.in_dc.ctypes.data
        self.in_base = (base + 4095) & ~4095
        assert self.svc.add_region(0, self.in_base, n_rec * 32 * CHUNK) == 0
        assert self.svc.add_region(1, self.lines, depth * 32) == 0
        self.tiles = []
        for c in range(clients):
            t = vtile.VTile(service=self.svc, client=c, seed=(seeds or [0x5eed + c] * clients)[c], **opts)
            assert t.set_svc_region(0, self.in_base, n_rec * 32 * CHUNK) == 0
            assert t.set_svc_region(1, self.lines, depth * 32) == 0
            if zero_copy:
                assert t.set_in_links([self.mc]) == 0
            self.tiles.append(t)
        self.next_chunk = 0

    def put(self, seq: int, payload: bytes) -> tuple[int, int]:
        """The producer: the record into the in dcache, then seq published on the mcache.  (addr, sz)"""
        rec = vtile.frag_bytes(payload)
        c = self.next_chunk
        self.next_chunk += (len(rec) + 2 * CHUNK - 1) // (2 * CHUNK) * 2
        off = self.in_base - self.in_dc.ctypes.data + c * CHUNK
        self.in_dc[off:off + len(rec)] = np.frombuffer(rec, np.uint8)
        self.L.fdgpu_mcache_publish(self.mc, seq, 0, c, len(rec), 0, 0)
        return self.in_base + c * CHUNK, len(rec)


def test_served_tile_attach_once():
    svc = vtile.Service(None, create=True, clients=2, batch_txn=1024)
    t0 = vtile.VTile(service=svc, client=0)
    with pytest.raises(RuntimeError):
        vtile.VTile(service=svc, client=0)          # a client slot takes one tile
    with pytest.raises(RuntimeError):
        vtile.VTile(service=svc, client=2)          # out of range
    t1 = vtile.VTile(service=svc, client=1)
    t0.close(); t1.close(); svc.close()


def test_served_zero_copy_results_in_order():
    rig = Rig()
    t = rig.tiles[0]
    pays = [_payload(i) for i in range(40)]
    pays[7] = pays[3]                                # a duplicate signature: dedup
    addrs = [rig.put(s, p) for s, p in enumerate(pays)]
    for s, (a, n) in enumerate(addrs):
        assert t.during_frag_at(a, n, s) == 0
    assert t.pending() == 40
    t.housekeep()                                    # publishes the requests
    # codes by request index: 5 -> ERR_SIG, 9 -> parse failure, the rest valid
    codes = np.zeros(40, np.int32)
    codes[5] = -1
    codes[9] = -16
    assert rig.svc.debug_serve(codes, FP) == 40
    n_left, _ = t.copy_state(0)
    out = t.after_frags(4096)
    t.housekeep()
    assert t.copy_state(0)[0] == 0                   # every frag copied: the link's credit may pass them
    assert [d[0] for d in out] == list(range(40))    # frag order
    res = [d[1] for d in out]
    want = [vtile.PUBLISH] * 40
    want[5], want[9], want[7] = vtile.VERIFY_FAIL, vtile.PARSE_FAIL, vtile.DEDUP_FAIL
    assert res == want
    for s, (seq, r, chunk, sz, tag, _) in enumerate(out):
        if r != vtile.PUBLISH:
            continue
        rec = t.record(chunk, 80 + len(pays[s]))
        assert rec[80:] == pays[s] and rec[:8] == bytes(8)
        assert int.from_bytes(rec[10:12], "little") == FP                  # txn_t_sz as the GPU writes it
        assert sz == ((80 + len(pays[s]) + 1) & ~1) + FP                  # fd_txn_m_realized_footprint
        assert tag == vtile.dedup_tag(0x5eed, pays[s][1:65])
    assert t.metrics() == [1, 1, 1, 0, 37]           # parse, verify, dedup, bundle peer, published


def test_served_overrun_at_copy():
    rig = Rig(depth=64)
    t = rig.tiles[0]
    a, n = rig.put(0, _payload(0))
    assert t.during_frag_at(a, n, 0) == 0
    rig.L.fdgpu_mcache_publish(rig.mc, 64, 0, 0, n, 0, 0)   # the producer laps the line before the copy
    t.housekeep()
    rig.svc.debug_serve(np.zeros(1, np.int32), FP)
    out = t.after_frags(16)
    assert [d[1] for d in out] == [vtile.OVERRUN] and t.overruns() == 1


def test_served_host_copy_and_two_tiles():
    rig = Rig(clients=2, zero_copy=False, seeds=[11, 22])
    pays = [_payload(100 + i) for i in range(30)]
    for s, p in enumerate(pays):                     # round robin over the two tiles; the tiles copy the frag
        assert rig.tiles[s % 2].during_frag(vtile.frag_bytes(p), s) == 0
    for t in rig.tiles:
        t.flush()
    codes = np.zeros(64, np.int32)
    codes[3] = -3                                    # request 3 of each tile: ERR_MSG
    assert rig.svc.debug_serve(codes, FP) == 30
    for k, t in enumerate(rig.tiles):
        out = t.after_frags(64, blocking=True)
        assert [d[0] for d in out] == list(range(k, 30, 2))
        assert [d[1] for d in out] == [vtile.VERIFY_FAIL if i == 3 else vtile.PUBLISH for i in range(15)]
        for (seq, r, chunk, sz, tag, _) in out:
            if r == vtile.PUBLISH:
                assert tag == vtile.dedup_tag([11, 22][k], pays[seq][1:65])   # each tile's own seed
                assert t.record(chunk, 80 + 200)[80:] == pays[seq]


def test_served_fault_completions():
    rig = Rig()
    t = rig.tiles[0]
    for s in range(6):
        a, n = rig.put(s, _payload(s))
        assert t.during_frag_at(a, n, s) == 0
    t.housekeep()
    codes = np.array([0, 0, -128, -128, 0, 0], np.int32)   # VSVC_CODE_FAULT: the service's batch failed
    rig.svc.debug_serve(codes, FP)
    out = t.after_frags(16)
    assert [d[1] for d in out] == [vtile.PUBLISH] * 2 + [vtile.GPU_FAULT] * 2 + [vtile.PUBLISH] * 2
    assert t.gpu_metrics()["gpu_fault_frags"] == 2


def test_served_service_gone():
    """A blocking drain never hangs on a service that stopped: once its heartbeat is older than 3 s the
    pending frags come back as GPU_FAULT, in order."""
    rig = Rig()
    t = rig.tiles[0]
    for s in range(3):
        a, n = rig.put(s, _payload(s))
        assert t.during_frag_at(a, n, s) == 0
    t.housekeep()
    rig.svc.debug_serve(np.zeros(1, np.int32), FP)   # serves the first three, beats once
    assert [d[1] for d in t.after_frags(16)] == [vtile.PUBLISH] * 3
    a, n = rig.put(3, _payload(3))
    assert t.during_frag_at(a, n, 3) == 0
    t0 = time.monotonic()
    out = t.after_frags(16, blocking=True)           # the service never comes back
    assert time.monotonic() - t0 < 10
    assert [(d[0], d[1]) for d in out] == [(3, vtile.GPU_FAULT)]
    assert t.faulted() >= 1


def _fake_sysfs(root, gpus):
    """gpus: [(location_id, domain, numa_node)]; node 0 is a CPU node"""
    topo = os.path.join(root, "class/kfd/kfd/topology/nodes")
    os.makedirs(os.path.join(topo, "0"))
    open(os.path.join(topo, "0/properties"), "w").write("cpu_cores_count 64\nsimd_count 0\n")
    for i, (loc, dom, node) in enumerate(gpus):
        d = os.path.join(topo, str(i + 1))
        os.makedirs(d)
        open(os.path.join(d, "properties"), "w").write(f"simd_count 1024\nlocation_id {loc}\ndomain {dom}\n")
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        p = os.path.join(root, "bus/pci/devices", bdf)
        os.makedirs(p)
        open(os.path.join(p, "numa_node"), "w").write(f"{node}\n")


def test_gpu_numa_node_sysfs(tmp_path, monkeypatch):
    """HIP device -> NUMA node without a GPU call: the device-th GPU of the KFD topology after
    ROCR_VISIBLE_DEVICES then HIP_VISIBLE_DEVICES, its PCI function's numa_node (the bench's host plan and
    the link's CPU choice use this; tests/test_gpu_vsvc.py checks it against the HIP device's bus id)."""
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    root = str(tmp_path)
    _fake_sysfs(root, [(0x0500, 0, 0), (0x1500, 0, 0), (0x8500, 0, 1), (0x9500, 1, 1)])
    assert [vtile.gpu_numa_node(d, root) for d in range(5)] == [0, 0, 1, 1, -1]
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "2,0")
    assert [vtile.gpu_numa_node(d, root) for d in range(3)] == [1, 0, -1]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert vtile.gpu_numa_node(0, root) == 0 and vtile.gpu_numa_node(1, root) == -1
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    assert vtile.gpu_numa_node(0, root) == 1
    assert vtile.gpu_numa_node(0, str(tmp_path / "none")) == -1


def test_served_request_outside_its_regions_is_refused():
    """A frag whose record lies outside every region the service registered is refused by the tile (-3) and
    never becomes a request; the service bounds every request it takes against its regions as well, so a
    hostile tile process cannot make the GPU read or write outside them (fdgpu_vsvc_poll)."""
    rig = Rig()
    t = rig.tiles[0]
    a, n = rig.put(0, _payload(0))
    assert t.during_frag_at(a, n, 0) == 0
    assert t.during_frag_at(rig.in_base + rig.in_dc.size - 4096 - 64, n, 1) == -3
    assert t.pending() == 1
    t.housekeep()
    assert rig.svc.debug_serve(np.zeros(1, np.int32), FP) == 1
    assert [d[1] for d in t.after_frags(16)] == [vtile.PUBLISH]


def test_service_ignores_a_rewritten_layout():
    """The segment is writable by every tile process, so the service takes no size or offset from it: it serves
    from the layout it made (fdgpu_vsvc_t's private copy).  A tile rewriting the header's client count and
    sizes, and its own ring and out-dcache offsets, changes nothing the service reads or writes."""
    rig = Rig()
    t = rig.tiles[0]
    pays = [_payload(300 + i) for i in range(8)]
    for s, p in enumerate(pays):
        a, n = rig.put(s, p)
        assert t.during_frag_at(a, n, s) == 0
    t.housekeep()
    h = ctypes.c_uint64.from_address(rig.svc.p).value          # fdgpu_vsvc_t.h: the shared header
    u64 = lambda off: ctypes.c_uint64.from_address(h + off)
    cl0 = 256                                                   # client[0] (64-aligned after rgn_sz[16])
    assert u64(cl0 + 144).value != u64(cl0 + 128).value         # off_out, off_req as made
    ctypes.c_int32.from_address(h + 16).value = 16              # clients
    u64(24).value = 1 << 40                                     # ring_cap
    u64(32).value = 1 << 50                                     # out_sz
    u64(cl0 + 136).value = u64(cl0 + 144).value                 # off_cpl -> the out dcache
    u64(cl0 + 144).value = u64(cl0 + 128).value                 # off_out -> the request ring
    u64(cl0 + 152).value = 1 << 40                              # ring_cap
    u64(cl0 + 160).value = 1 << 50                              # out_sz
    assert rig.svc.debug_serve(np.zeros(8, np.int32), FP) == 8
    out = t.after_frags(64)
    assert [(d[0], d[1]) for d in out] == [(s, vtile.PUBLISH) for s in range(8)]
    for s, (seq, r, chunk, sz, tag, _) in enumerate(out):
        assert t.record(chunk, 80 + len(pays[s]))[80:] == pays[s]
        assert tag == vtile.dedup_tag(0x5eed, pays[s][1:65])
