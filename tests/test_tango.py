"""CPU: the host-only pieces of the GPU verify tile (libfdgpu_vtile.so):
the HA dedup tag (XXH64, checked against the xxhash package), the tcache
against a model of FD_TCACHE_QUERY / FD_TCACHE_INSERT
(src/tango/tcache/fd_tcache.h:281-404), mcache publish / poll incl.
overrun, and fd_dcache_compact_next."""
import collections
import ctypes

import numpy as np
import pytest

from firedancer_amd import vtile


def test_exports():
    L = vtile.load()
    for name in vtile.EXPORTS:
        assert hasattr(L, name), name


def test_dedup_tag_is_xxh64():
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(3)
    for _ in range(200):
        sig, seed = rng.bytes(64), int(rng.integers(0, 2**63))
        assert vtile.dedup_tag(seed, sig) == xxhash.xxh64(sig, seed=seed).intdigest()


class TCacheModel:
    def __init__(self, depth):
        self.depth, self.ring, self.set = depth, collections.deque(), set()

    def query(self, tag):
        return tag == 0 or tag in self.set

    def insert(self, tag):
        if self.query(tag):
            return True
        self.ring.append(tag); self.set.add(tag)
        if len(self.ring) > self.depth:
            self.set.discard(self.ring.popleft())
        return False


@pytest.mark.parametrize("depth", [1, 2, 7, 64, 1000])
def test_tcache_vs_model(depth):
    rng = np.random.default_rng(depth)
    tc, m = vtile.TCache(depth), TCacheModel(depth)
    universe = rng.integers(1, 2**63, max(4, 3 * depth), dtype=np.uint64)
    for i in range(20000):
        tag = int(universe[rng.integers(len(universe))]) if i % 50 else 0
        if rng.integers(3):
            assert tc.insert(tag) == m.insert(tag), i
        else:
            assert tc.query(tag) == m.query(tag), i


def test_tcache_probe_chains_survive_eviction():
    # tags that collide in the map exercise the backward-shift delete
    tc, m = vtile.TCache(16), TCacheModel(16)
    tags = [(k << 40) | 1 for k in range(1, 400)]
    for i, t in enumerate(tags * 3):
        assert tc.insert(t) == m.insert(t)
        for q in tags[max(0, i % len(tags) - 20): i % len(tags) + 1]:
            assert tc.query(q) == m.query(q)


def test_mcache_publish_poll_overrun():
    L = vtile.load()
    mc = L.fdgpu_mcache_new(8, 100)
    meta = vtile.FragMeta()
    assert L.fdgpu_mcache_poll(mc, 100, ctypes.byref(meta)) == 1          # not yet published
    for s in range(100, 110):
        L.fdgpu_mcache_publish(mc, s, s * 3, s % 7, 1000 + s, s + 1, s + 2)
    assert L.fdgpu_mcache_poll(mc, 105, ctypes.byref(meta)) == 0
    assert (meta.seq, meta.sig, meta.chunk, meta.sz, meta.tsorig) == (105, 315, 0, 1105, 106)
    assert L.fdgpu_mcache_poll(mc, 101, ctypes.byref(meta)) == -1         # lapped by 109
    assert L.fdgpu_mcache_poll(mc, 110, ctypes.byref(meta)) == 1
    L.fdgpu_mcache_delete(mc)


def test_dcache_compact_next():
    L = vtile.load()
    # advances in 128-byte chunk pairs, wraps to chunk0 past wmark (fd_dcache.h:263-269)
    assert L.fdgpu_dcache_compact_next(10, 1, 10, 100) == 12
    assert L.fdgpu_dcache_compact_next(10, 128, 10, 100) == 12
    assert L.fdgpu_dcache_compact_next(10, 129, 10, 100) == 14
    assert L.fdgpu_dcache_compact_next(98, 1312, 10, 100) == 10


def test_xxh64_any_length():
    """fdgpu_xxh64 (the link's verdict trace hashes published records with it) is XXH64"""
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(4)
    for n in list(range(0, 80)) + [255, 1312, 2087]:
        data, seed = rng.bytes(n), int(rng.integers(0, 2**63))
        assert vtile.xxh64(seed, data) == xxhash.xxh64(data, seed=seed).intdigest(), n
