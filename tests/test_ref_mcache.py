"""CPU: the tile reads the reference's own mcache.  A ring of fd_frag_meta_t lines is initialised and
written by the reference's producer code (fd_mcache_publish / fd_mcache_publish_avx, compiled in place
into oracle/_ref/libfdref_mcache.so) and read through fdgpu_mcache_wrap (include/fd_verify_gpu.h) --
the handle the GPU tile's zero-copy intake re-checks lines through.  Every read must agree with the
reference consumer, FD_MCACHE_WAIT, on the same ring: the metadata of a published frag, "not yet" for a
future seq, "overrun" with the same seq_found once the producer has lapped it, across the 2^64 seq wrap
(the full 64-bit seqs the stem hands the tile, fd_stem.c:627,668,700)."""
import ctypes

import numpy as np
import pytest

from firedancer_amd import vtile


def _ref(depth, seq0):
    from oracle.oracle import RefMcache
    try:
        return RefMcache(depth, seq0)
    except FileNotFoundError as e:
        pytest.skip(f"reference mcache build unavailable: {e}")


def _query(L, mc, seq):
    m = vtile.FragMeta()
    found = ctypes.c_ulong(0)
    rc = L.fdgpu_mcache_query(mc, seq, ctypes.byref(m), ctypes.byref(found))
    return rc, m, int(found.value)


@pytest.mark.parametrize("seq0", [0, 12345, (1 << 64) - 40])
@pytest.mark.parametrize("avx", [False, True])
def test_wrap_reads_reference_published_lines(seq0, avx):
    depth = 64
    ref = _ref(depth, seq0)
    L = vtile.load()
    mc = L.fdgpu_mcache_wrap(ref.lines_addr, depth)
    assert mc and L.fdgpu_mcache_depth(mc) == depth and L.fdgpu_mcache_lines(mc) == ref.lines_addr
    M = (1 << 64) - 1
    rng = np.random.default_rng(seq0 & 0xffff)
    n = 3 * depth + 7
    pub = {}
    for i in range(n):
        seq = (seq0 + i) & M
        f = dict(sig=int(rng.integers(0, 1 << 63)), chunk=int(rng.integers(0, 1 << 31)), sz=int(rng.integers(0, 1 << 16)),
                 ctl=int(rng.integers(0, 1 << 16)), tsorig=int(rng.integers(0, 1 << 32)), tspub=int(rng.integers(0, 1 << 32)))
        # before the publish: not yet (both consumers)
        rc_r, _, _ = ref.wait(seq)
        rc_g, _, _ = _query(L, mc, seq)
        assert rc_r == rc_g == 1
        ref.publish(seq, avx=avx, **f)
        pub[seq] = f
        assert ref.line_idx(seq) == seq & (depth - 1)
        # every seq still in the ring reads as the reference reads it; lapped ones as overruns
        for back in (0, 1, depth - 1, depth, depth + 3):
            if back > i:
                continue
            s = (seq - back) & M
            rc_r, meta, found_r = ref.wait(s)
            rc_g, m, found_g = _query(L, mc, s)
            assert rc_g == rc_r, (i, back)
            assert found_g == found_r
            if rc_r == 0:
                want = pub[s]
                assert (m.seq, m.sig, m.chunk, m.sz, m.tsorig, m.tspub) == (
                    s, want["sig"], want["chunk"], want["sz"], want["tsorig"], want["tspub"])
                assert int(meta["seq"]) == s and int(meta["ctl"]) == want["ctl"]
            else:
                assert rc_r == -1 and back >= depth
    # the handle wrote nothing: the lines are still exactly what the reference published
    for i in range(n - depth, n):
        s = (seq0 + i) & M
        ln = ref.lines[ref.line_idx(s)]
        assert int(ln["seq"]) == s and int(ln["sig"]) == pub[s]["sig"] and int(ln["sz"]) == pub[s]["sz"]
    L.fdgpu_mcache_delete(mc)


def test_wrap_rejects_bad_rings():
    L = vtile.load()
    buf = np.zeros(4096 + 64, np.uint8)
    a = buf.ctypes.data + ((-buf.ctypes.data) % 64)
    assert not L.fdgpu_mcache_wrap(a, 48)              # depth not a power of 2
    assert not L.fdgpu_mcache_wrap(a + 8, 64)          # lines not 32-byte aligned
    assert not L.fdgpu_mcache_wrap(None, 64)
    mc = L.fdgpu_mcache_wrap(a, 64)
    assert mc
    L.fdgpu_mcache_delete(mc)


def test_stem_consumer_over_reference_ring():
    """A stem-shaped consumer (fd_stem.c:570-700: poll the next seq; on an overrun resume at seq_found)
    over the wrapped reference ring with a producer that laps it: the frags the consumer takes are
    exactly the ones FD_MCACHE_WAIT takes, in order, and every skipped seq is accounted as lost."""
    depth = 32
    ref = _ref(depth, 7)
    L = vtile.load()
    mc = L.fdgpu_mcache_wrap(ref.lines_addr, depth)
    rng = np.random.default_rng(3)
    prod, cons_g, cons_r = 7, 7, 7
    took_g, took_r, lost_g, lost_r = [], [], 0, 0
    for step in range(4000):
        for _ in range(int(rng.integers(0, 3 * depth // 2))):     # a bursty producer that sometimes laps
            ref.publish(prod, sig=prod * 3, chunk=prod % 1000, sz=64 + prod % 1000)
            prod += 1
        for _ in range(int(rng.integers(0, depth))):
            rc, m, found = _query(L, mc, cons_g)
            if rc == 1:
                break
            if rc < 0:
                lost_g += found - cons_g
                cons_g = found
                continue
            took_g.append((m.seq, m.sig, m.chunk, m.sz))
            cons_g += 1
        for _ in range(int(rng.integers(0, depth))):
            rc, meta, found = ref.wait(cons_r)
            if rc == 1:
                break
            if rc < 0:
                lost_r += found - cons_r
                cons_r = found
                continue
            took_r.append((int(meta["seq"]), int(meta["sig"]), int(meta["chunk"]), int(meta["sz"])))
            cons_r += 1
    assert lost_g > 0 and len(took_g) > 1000
    assert all(t == (s, s * 3, s % 1000, 64 + s % 1000) for t in took_g for s in [t[0]])
    assert [t[0] for t in took_g] == sorted(t[0] for t in took_g)
    assert len(took_g) + lost_g == cons_g - 7
    assert len(took_r) + lost_r == cons_r - 7
    L.fdgpu_mcache_delete(mc)
