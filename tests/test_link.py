"""CPU: the configs[4] link (fd_verify_gpu.c) without a GPU.

* The verify-tile -> GPU binding: tile i takes seq % T == i
  (fd_verify_tile.c:47-48) and drives GPU i % G in that GPU's process.
* A link created in one process and joined from another: the same
  configuration, the prefilled in dcache (one fd_txn_m_t record per
  distinct payload), and mcache lines published in one process polled in
  the other -- including the overrun a lapped consumer sees on an
  unreliable link.
"""
import ctypes
import multiprocessing as mp
import os
import tempfile

import numpy as np
import pytest

from firedancer_amd import vtile


@pytest.mark.parametrize("tiles,gpus", [(1, 1), (6, 1), (2, 2), (6, 4), (16, 8), (48, 8)])
def test_tile_device_binding(tiles, gpus):
    per = [vtile.tiles_of(tiles, gpus, g) for g in range(gpus)]
    assert sorted(sum(per, [])) == list(range(tiles))            # every tile runs exactly once
    for g, ts in enumerate(per):
        assert ts == [i for i in range(tiles) if i % gpus == g]  # tile i -> GPU i mod G
    assert vtile.tiles_of(tiles, gpus, gpus) == [] and vtile.tiles_of(tiles, gpus, -1) == []


def test_tile_device_binding_examples():
    assert vtile.tiles_of(6, 1, 0) == [0, 1, 2, 3, 4, 5]
    assert vtile.tiles_of(16, 8, 3) == [3, 11]
    assert [vtile.tiles_of(6, 4, g) for g in range(4)] == [[0, 4], [1, 5], [2], [3]]


def _payloads(n=5):
    rng = np.random.default_rng(1)
    sz = np.array([1232, 7, 300, 1, 1000][:n], np.uint16)
    off = np.concatenate([[0], np.cumsum(sz)[:-1]]).astype(np.uint32)
    payload = rng.integers(0, 256, int(sz.sum()), dtype=np.uint8)
    return payload, off, sz


def _shm_dir():
    return "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()


def _joiner(path, q, back):
    from firedancer_amd import vtile as vt
    L = vt.load()
    link = vt.Link(path, create=False, timeout_s=30)
    cfg = link.cfg()
    mc = link.mcache()
    meta = vt.FragMeta()
    polls = [L.fdgpu_mcache_poll(ctypes.c_void_p(mc), s, ctypes.byref(meta)) for s in range(4)]
    first = (meta.seq, meta.chunk, meta.sz) if polls[-1] == 0 else None
    recs = [ctypes.string_at(link.dcache() + 64 * c, 16) for c in (0, 22)]
    q.put((cfg, polls, first, link.joined(), recs))
    back.get(timeout=60)                                     # wait: the parent publishes a lap
    q.put(L.fdgpu_mcache_poll(ctypes.c_void_p(mc), 0, ctypes.byref(meta)))
    link.close()


def test_link_shared_between_processes():
    payload, off, sz = _payloads()
    path = os.path.join(_shm_dir(), f"fdgpu_link_test_{os.getpid()}")
    link = vtile.Link(path, create=True, payload=payload, off=off, sz=sz, n_frags=1000, tiles=6, gpus=2,
                      batch_txn=512, rate_fps=1e6, zero_copy=True, reliable=False, mcache_depth=64)
    try:
        L = vtile.load()
        mc = link.mcache()
        for s in range(4):                                   # seq s -> payload s % 5, as the producer publishes
            L.fdgpu_mcache_publish(ctypes.c_void_p(mc), s, 0, 0 if s == 0 else 22, 80 + int(sz[s]), 1000 + s, 1000 + s)
        ctx = mp.get_context("spawn")
        q, back = ctx.Queue(), ctx.Queue()
        p = ctx.Process(target=_joiner, args=(path, q, back), daemon=True)
        p.start()
        cfg, polls, first, joined, recs = q.get(timeout=60)
        os.unlink(path)                                      # every process has it mapped: the file can go
        assert cfg["tiles"] == 6 and cfg["gpus"] == 2 and cfg["reliable"] == 0 and cfg["n_frags"] == 1000
        assert cfg["batch_txn"] == 512 and cfg["zero_copy"] == 1 and abs(cfg["rate_fps"] - 1e6) < 1e-6
        assert polls == [0, 0, 0, 0] and first == (3, 22, 81) and joined == 2
        # the in dcache holds fd_txn_m_t records: payload_sz at byte 8 of the header
        assert int.from_bytes(recs[0][8:10], "little") == 1232
        # record 1 (7-byte payload) sits at the chunk after record 0's 1312 bytes -> 22
        assert int.from_bytes(recs[1][8:10], "little") == 7
        for s in range(4, 64 + 1):                           # a full lap: line 0 now holds seq 64
            L.fdgpu_mcache_publish(ctypes.c_void_p(mc), s, 0, 0, 0, 0, 0)
        back.put("go")
        assert q.get(timeout=60) == -1                       # the joiner polling seq 0 is overrun
        p.join(timeout=60)
        assert p.exitcode == 0
    finally:
        link.close()
        if os.path.exists(path):
            os.unlink(path)


def test_link_rejects_bad_config():
    payload, off, sz = _payloads()
    with pytest.raises(RuntimeError):
        vtile.Link(None, create=True, payload=payload, off=off, sz=sz, n_frags=10, tiles=2, gpus=3)   # G > T
    with pytest.raises(RuntimeError):
        vtile.Link(None, create=True, payload=payload, off=off, sz=sz, n_frags=10, tiles=65, gpus=1)
    big = np.array([1233], np.uint16)
    with pytest.raises(RuntimeError):
        vtile.Link(None, create=True, payload=np.zeros(1233, np.uint8), off=np.zeros(1, np.uint32), sz=big,
                   n_frags=10, tiles=1, gpus=1)
    with pytest.raises(RuntimeError):
        vtile.Link(os.path.join(_shm_dir(), "fdgpu_link_absent"), create=False, timeout_s=0.05)


def test_link_producers_config():
    """Q producer links (the reference's QUIC tiles): the count travels in the shared configuration;
    the default is one; more than FDGPU_VTILE_IN_MAX (16) is refused."""
    payload, off, sz = _payloads()
    link = vtile.Link(None, create=True, payload=payload, off=off, sz=sz, n_frags=100, tiles=4, gpus=2, producers=3)
    try:
        assert link.cfg()["producers"] == 3 and link.mcache()
    finally:
        link.close()
    link = vtile.Link(None, create=True, payload=payload, off=off, sz=sz, n_frags=100, tiles=2, gpus=1)
    try:
        assert link.cfg()["producers"] == 1
    finally:
        link.close()
    with pytest.raises(RuntimeError):
        vtile.Link(None, create=True, payload=payload, off=off, sz=sz, n_frags=10, tiles=2, gpus=1, producers=17)
