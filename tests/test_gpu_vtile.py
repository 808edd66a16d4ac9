"""GPU: the verify tile over the engine (libfdgpu_vtile.so) against the
reference tile's own per-frag decision (oracle/_ref/libfdref_tile.so:
fd_txn_verify, the tcache, fd_hash, fd_txn_parse and the AVX-512 verify
compiled in place from the reference, src/disco/verify/fd_verify_tile.c:
103-157 + fd_verify_tile.h:59-108): same per-frag outcome, same metrics,
same published fd_txn_m_t records (payload + fd_txn_t image) and same HA
dedup tags, over a stream with valid / invalid signatures, parse
failures, HA duplicates (incl. tcache eviction) and bundles with failing
members.  Without the reference build, the sequential model below (which
tests/test_ref_tile.py pins to it) is the expectation."""
import ctypes
import os
import sys
import time

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import raw_expect  # noqa: E402
import txn_builder as tb  # noqa: E402
from test_tango import TCacheModel  # noqa: E402

pytestmark = pytest.mark.gpu


def make_stream(seed=11):
    from firedancer_amd import synth
    rng = np.random.default_rng(seed)
    base = []
    for kind, ms, inv, n, s in ((synth.LARGE_NOOP, 1, 0.0, 300, 1), (synth.MULTI, 12, 0.25, 200, 2),
                                (synth.SMALL_MSG, 1, 0.1, 100, 3)):
        payload, desc, _, _ = synth.make_batch(n, kind, ms, inv, seed=s)
        base += [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    base += [tb.build_txn(rng) for _ in range(60)]
    base += [tb.mutate(rng, base[int(rng.integers(600))]) for _ in range(60)]
    base = [b for b in base if len(b) <= 1232]          # the tile FD_LOG_ERRs on > FD_TPU_MTU (fd_verify_tile.c:83-85)
    order = list(rng.permutation(len(base)))
    frags, bid = [], 0
    i = 0
    while i < len(order):
        r = rng.random()
        if r < 0.15:                                   # HA duplicate of something seen earlier
            j = int(rng.integers(max(1, len(frags))))
            frags.append((frags[j][0] if frags else base[order[i]], 0))
        elif r < 0.25:                                 # a bundle of 2..5 frags
            bid += 1
            for _ in range(int(rng.integers(2, 6))):
                if i < len(order):
                    frags.append((base[order[i]], 1000 + bid)); i += 1
            continue
        else:
            frags.append((base[order[i]], 0))
        i += 1
    return frags


def model(oracle, frags, seed, depth):
    from firedancer_amd import vtile
    import xxhash
    arena, off, sz = tb.pack([p for p, _ in frags])
    codes, fp, img = raw_expect.expected_codes(oracle, arena, off, sz)
    tc, bundle_failed, bundle_id = TCacheModel(depth), 0, 0
    res, metrics, recs = [], [0] * 5, {}
    for i, (p, b) in enumerate(frags):
        is_bundle = b != 0
        if is_bundle and b != bundle_id:
            bundle_failed, bundle_id = 0, b
        if is_bundle and bundle_failed:
            metrics[3] += 1; res.append(vtile.BUNDLE_PEER_FAIL); continue
        if fp[i] == 0:
            bundle_failed |= is_bundle; metrics[0] += 1; res.append(vtile.PARSE_FAIL); continue
        so = int(img[i, 2]) | int(img[i, 3]) << 8
        tag = xxhash.xxh64(p[so: so + 64], seed=seed).intdigest()
        if not is_bundle and tc.query(tag):
            r = vtile.DEDUP_FAIL
        elif codes[i] != 0:
            r = vtile.VERIFY_FAIL
        elif not is_bundle and tc.insert(tag):
            r = vtile.DEDUP_FAIL
        else:
            r = vtile.PUBLISH
        if r != vtile.PUBLISH:
            bundle_failed |= is_bundle
            metrics[2 if r == vtile.DEDUP_FAIL else 1] += 1
        else:
            metrics[4] += 1
            h = np.frombuffer(vtile.frag_bytes(p, b), np.uint8).copy()
            h[10:12] = np.frombuffer(np.uint16(fp[i]).tobytes(), np.uint8)   # txn_t_sz
            recs[i] = (h.tobytes(), img[i, : fp[i]].tobytes())   # the alignment pad byte between them is unspecified
        res.append(r)
    return res, metrics, recs


def expectation(oracle, frags, seed, depth):
    """(per-frag results, metrics, {i: (record head, fd_txn_t bytes)}, {i: tag}) of the reference tile."""
    from oracle.oracle import RefTile
    try:
        ref = RefTile()
    except (FileNotFoundError, RuntimeError):
        res, m, recs = model(oracle, frags, seed, depth)
        return res, m, recs, None
    res, m, recs, tags = ref.run(frags, depth, seed)
    out = {}
    for i, r in recs.items():
        hl = 80 + len(frags[i][0])
        out[i] = (r[:hl], r[(hl + 1) & ~1:])
    return res, m, out, {i: tags[i] for i in recs}


def in_dcache(frag_list):
    """The frags as fd_txn_m_t records in one 64-B-chunked in dcache (numpy, page-locked by the caller)."""
    offs, pos = [], 0
    for fb in frag_list:
        offs.append(pos)
        pos += (len(fb) + 63) & ~63
    buf = np.zeros(pos + 4096 + 128, np.uint8)
    base = (-buf.ctypes.data) % 64                       # chunk-align the first record
    for fb, o in zip(frag_list, offs):
        buf[base + o: base + o + len(fb)] = np.frombuffer(fb, np.uint8)
    return buf, [base + o for o in offs]


@pytest.mark.parametrize("zero_copy", [False, True, "finish", "host"])
@pytest.mark.parametrize("batch,depth", [(64, 32), (512, 1 << 12)])
def test_vtile_vs_model(oracle, batch, depth, zero_copy, engine_path):
    """zero_copy: the frags stay in a registered in dcache and the GPU gathers them into the out
    dcache records (fdgpu_vtile_set_in_link); outcomes and published records must not change.
    "finish": the same, with the records written into the out dcache by each batch's fd_finish_kernel
    from the device arena instead of by the gather kernel (fdgpu_debug_opts_t.gather_no_writeback = 2).
    "host": the GPU copy only reads each record; two host copy threads of the tile write it into the out
    dcache (fdgpu_vtile_opts_t.copy_threads, FDGPU_GATHER_NO_WRITEBACK)."""
    pytest.importorskip("xxhash")
    from firedancer_amd import engine, vtile
    if zero_copy == "finish":
        from conftest import engine_opts
        engine.debug_set_opts(**engine_opts(engine_path, gather_no_writeback=2))
    frags = make_stream()
    seed = 0x1234abcd
    want_res, want_m, want_recs, want_tags = expectation(oracle, frags, seed, depth)
    vt = vtile.VTile(device=0, batch_txn=batch, tcache_depth=depth, seed=seed,
                     copy_threads=2 if zero_copy == "host" else 0)
    if zero_copy:
        fbs = [vtile.frag_bytes(p, b) for p, b in frags]
        buf, offs = in_dcache(fbs)
        engine.host_register(buf)
        assert vt.set_in_link(None) == 0
    got, bad = [], []

    def drain(blocking):
        # downstream reads each published record as it is published (the out dcache is a ring)
        out = vt.after_frags(blocking=blocking)
        for seq, r, chunk, sz, tag, _ in out:
            if r == vtile.PUBLISH:
                head, timg = want_recs.get(seq, (b"", b""))
                rec = vt.record(chunk, sz)
                if rec[: len(head)] != head or rec[(len(head) + 1) & ~1:] != timg or sz != ((len(head) + 1) & ~1) + len(timg):
                    bad.append(seq)
                if want_tags is not None and tag != want_tags.get(seq):
                    bad.append(("tag", seq))
        return out

    for seq, (p, b) in enumerate(frags):
        fb = vtile.frag_bytes(p, b)
        while True:
            rc = vt.during_frag_at(buf.ctypes.data + offs[seq], len(fb), seq) if zero_copy else vt.during_frag(fb, seq)
            if rc != -2:
                break
            got += drain(True)
        assert rc == 0, rc
        if seq % 37 == 0:
            got += drain(False)
    vt.flush()
    while vt.pending():
        got += drain(True)
    assert [g[0] for g in got] == list(range(len(frags)))
    assert [g[1] for g in got] == want_res
    assert vt.metrics() == want_m
    assert bad == []
    assert sum(want_m[:4]) > 100 and want_m[2] > 10 and want_m[3] > 0
    hc = vt.gpu_metrics()["host_copy"]
    assert (hc[0] == len(frags) and hc[2] == 0) if zero_copy == "host" else hc == [0, 0, 0, 0]
    vt.close()
    if zero_copy:
        engine.host_unregister(buf)


@pytest.mark.parametrize("launcher", [0, 1])
@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("nctx", [1, 2, 3])
def test_vtile_multictx_vs_model(oracle, nctx, zero_copy, launcher):
    """Adaptive batching over nctx engine contexts (fdgpu_vtile_opts_t) (housekeep launches batches into the
    contexts in turn, staggered): completions merged back into frag order must give exactly the
    model's per-frag outcomes, metrics and published records.  launcher: the contexts' launches and early
    copies made by the tile's launch thread (fdgpu_vtile_opts_t.launcher), the tile's thread only queueing."""
    pytest.importorskip("xxhash")
    from firedancer_amd import engine, vtile
    frags = make_stream(seed=12)
    seed, depth = 0x5eedbeef, 1 << 12
    want_res, want_m, want_recs, want_tags = expectation(oracle, frags, seed, depth)
    vt = vtile.VTile(device=0, batch_txn=128, tcache_depth=depth, seed=seed, nctx=nctx, launcher=launcher)
    if zero_copy:
        fbs = [vtile.frag_bytes(p, b) for p, b in frags]
        buf, offs = in_dcache(fbs)
        engine.host_register(buf)
        assert vt.set_in_link(None) == 0
    got, bad, launched = [], [], 0

    def drain(blocking):
        out = vt.after_frags(blocking=blocking)
        for seq, r, chunk, sz, tag, _ in out:
            if r == vtile.PUBLISH:
                head, timg = want_recs.get(seq, (b"", b""))
                rec = vt.record(chunk, sz)
                if rec[: len(head)] != head or rec[(len(head) + 1) & ~1:] != timg or sz != ((len(head) + 1) & ~1) + len(timg):
                    bad.append(seq)
                if want_tags is not None and tag != want_tags.get(seq):
                    bad.append(("tag", seq))
        return out

    for seq, (p, b) in enumerate(frags):
        fb = vtile.frag_bytes(p, b)
        while True:
            rc = vt.during_frag_at(buf.ctypes.data + offs[seq], len(fb), seq) if zero_copy else vt.during_frag(fb, seq)
            if rc != -2:
                break
            got += drain(True)
        assert rc == 0, rc
        if seq % 5 == 0:
            launched += vt.housekeep(1)
            time.sleep(3e-4)              # let batches finish between launches: many small staggered batches
        if seq % 11 == 0:
            got += drain(False)
    vt.flush()
    while vt.pending():
        got += drain(True)
    assert [g[0] for g in got] == list(range(len(frags)))
    assert [g[1] for g in got] == want_res
    assert vt.metrics() == want_m
    assert bad == []
    assert launched > 20
    lm = vt.gpu_metrics()["launcher"]
    assert (lm[0] >= launched) if launcher else not any(lm)
    vt.close()
    if zero_copy:
        engine.host_unregister(buf)


def _overrun_setup(n, depth, seed):
    from firedancer_amd import engine, synth, vtile
    L = vtile.load()
    payload, desc, _, _ = synth.make_batch(n, synth.LARGE_NOOP, seed=seed)
    fbs = [vtile.frag_bytes(payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes()) for d in desc]
    buf, offs = in_dcache(fbs)
    engine.host_register(buf)
    mc = L.fdgpu_mcache_new(depth, 0)
    for seq in range(n):
        L.fdgpu_mcache_publish(mc, seq, 0, seq, len(fbs[seq]), 0, 0)
    return L, fbs, buf, offs, mc


def _drain_all(vt):
    vt.flush()
    got = []
    while vt.pending():
        got += vt.after_frags(blocking=True)
    return got


def test_vtile_zero_copy_overrun():
    """Zero-copy intake, lap BEFORE the copy: the producer reuses the mcache lines of frags 0..23
    after during_frag took them but before the GPU copied them (the batch launch copies here).  The
    gather kernel re-reads each line right after its copy (the stem's seq / copy / re-check,
    fd_stem.c:667-686): those frags are OVERRUN, never parsed or published; the others publish."""
    from firedancer_amd import engine, vtile
    depth, n = 64, 64
    L, fbs, buf, offs, mc = _overrun_setup(n, depth, 21)
    vt = vtile.VTile(device=0, batch_txn=256, tcache_depth=1024)
    assert vt.set_in_link(mc) == 0
    for seq in range(n):
        assert vt.during_frag_at(buf.ctypes.data + offs[seq], len(fbs[seq]), seq) == 0
    assert vt.copy_state(0) == (n, 0)                  # nothing copied yet: a reliable credit would stop at 0
    for seq in range(n, n + 24):                       # the producer laps lines 0..23 before the copy
        L.fdgpu_mcache_publish(mc, seq, 0, 0, 0, 0, 0)
    got = _drain_all(vt)
    assert [g[0] for g in got] == list(range(n))
    assert [g[1] for g in got] == [vtile.OVERRUN] * 24 + [vtile.PUBLISH] * (n - 24)
    assert vt.overruns() == 24 and vt.metrics() == [0, 0, 0, 0, n - 24]
    assert vt.copy_state(0) == (0, n)
    vt.close()
    L.fdgpu_mcache_delete(mc)
    engine.host_unregister(buf)


def test_vtile_zero_copy_lap_after_copy():
    """Zero-copy intake, lap AFTER the copy: the reference decides an overrun once, right after
    during_frag's copy; a lap after that changes nothing (the out-dcache copy is what it publishes).
    Frags 0..31 are copied by the GPU (fdgpu_vtile_copy, waited for) before the producer laps lines
    0..39: they PUBLISH, bit for bit the reference's records; frags 32..39, taken but not yet
    copied when their lines were reused, are OVERRUN; 40..63 publish.  Round 2 checked at the
    verdict and dropped 0..31 too."""
    from firedancer_amd import engine, vtile
    depth, n = 64, 64
    L, fbs, buf, offs, mc = _overrun_setup(n, depth, 22)
    vt = vtile.VTile(device=0, batch_txn=256, tcache_depth=1024)
    assert vt.set_in_link(mc) == 0
    for seq in range(32):
        assert vt.during_frag_at(buf.ctypes.data + offs[seq], len(fbs[seq]), seq) == 0
    assert vt.copy(blocking=True) == 0
    assert vt.copy_state(0) == (0, 32)                 # 0..31 copied: a reliable credit may pass them
    for seq in range(32, n):
        assert vt.during_frag_at(buf.ctypes.data + offs[seq], len(fbs[seq]), seq) == 0
    assert vt.copy_state(0) == (32, 32)
    for seq in range(n, n + 40):                       # laps lines 0..39
        L.fdgpu_mcache_publish(mc, seq, 0, 0, 0, 0, 0)
    # the producer also rewrites the in-dcache bytes of frags 0..7 (their copies are already taken)
    for seq in range(8):
        buf[offs[seq] + 80: offs[seq] + 80 + 64] ^= 0xff
    got = _drain_all(vt)
    assert [g[0] for g in got] == list(range(n))
    want = [vtile.PUBLISH] * 32 + [vtile.OVERRUN] * 8 + [vtile.PUBLISH] * (n - 40)
    assert [g[1] for g in got] == want
    assert vt.overruns() == 8 and vt.metrics() == [0, 0, 0, 0, n - 8]
    for seq, r, chunk, sz, tag, _ in got[:8]:             # published records hold the bytes copied before the rewrite
        rec = vt.record(chunk, sz)
        assert rec[:len(fbs[seq])][80:] == fbs[seq][80:]
    vt.close()
    L.fdgpu_mcache_delete(mc)
    engine.host_unregister(buf)


@pytest.mark.parametrize("lap", [0, 24])
@pytest.mark.parametrize("rr_idx", [0, 1])
def test_vtile_on_reference_mcache(rr_idx, lap):
    """The tile bound to the reference's own tango shapes.  The in link's ring is an fd_frag_meta_t array
    written by the reference's fd_mcache_publish (oracle/_ref/libfdref_mcache.so, compiled in place) with
    seqs that cross 2^64, wrapped with fdgpu_mcache_wrap; the tile is driven as the stem drives it
    (fd_stem.c:627,668,700): before_frag( in_idx, seq, sig ) and during_frag_chunk( in_idx, seq, sig,
    chunk, sz, ctl ) on the line's fields, zero-copy intake from the registered in dcache with the GPU's
    line re-check.  Verify:rr_idx of 2 keeps every other frag (round robin on the full 64-bit seq); the
    kept frags' outcomes, records and HA tags equal the reference tile's, and each verdict carries its
    in_idx and full seq.  lap: the producer reuses the lines of the first `lap` seqs after the tile took
    them and before the GPU copied them -- those frags are OVERRUN and never reach after_frag, as in
    the reference."""
    pytest.importorskip("xxhash")
    from firedancer_amd import engine, vtile
    from oracle.oracle import RefMcache, RefTile
    try:
        ring, ref = RefMcache(256, (1 << 64) - 100), RefTile()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"reference build unavailable: {e}")
    M = (1 << 64) - 1
    seq0 = (1 << 64) - 100
    frags = make_stream(5)[:200]
    fbs = [vtile.frag_bytes(p, b) for p, b in frags]
    buf, offs = in_dcache(fbs)
    mem = buf.ctypes.data + offs[0]                     # chunk 0 of the link (64-B aligned)
    chunks = [(buf.ctypes.data + o - mem) // 64 for o in offs]
    engine.host_register(buf)
    L = vtile.load()
    mc = L.fdgpu_mcache_wrap(ring.lines_addr, ring.depth)
    depth, seed = 1 << 12, 0x5eed
    vt = vtile.VTile(device=0, batch_txn=256, tcache_depth=depth, seed=seed)
    vt.set_round_robin(rr_idx, 2)
    assert vt.set_in(0, vtile.IN_QUIC, mem, 0, max(chunks)) == 0
    assert vt.set_in_links([mc]) == 0
    assert vt.during_frag_chunk(0, seq0, 0, max(chunks) + 1, 100) == -4   # outside [chunk0, wmark]: corrupt
    for i, fb in enumerate(fbs):                        # the producer (the reference's publish)
        ring.publish((seq0 + i) & M, sig=0, chunk=chunks[i], sz=len(fb), ctl=0, tsorig=i, tspub=i)
    kept = []
    for i in range(len(fbs)):                           # the stem: poll the line, before_frag, during_frag
        s = (seq0 + i) & M
        m = vtile.FragMeta()
        assert L.fdgpu_mcache_poll(mc, s, m) == 0 and m.seq == s
        if vt.before_frag(0, s, m.sig):
            continue
        assert vt.during_frag_chunk(0, s, m.sig, m.chunk, m.sz, 0, m.tsorig) == 0
        kept.append(i)
    assert kept == [i for i in range(len(fbs)) if ((seq0 + i) & M) % 2 == rr_idx]
    for j in range(lap):                                # laps the lines of seqs seq0 .. seq0+lap-1
        ring.publish((seq0 + ring.depth + j) & M, sig=0, chunk=0, sz=0)
    got = _drain_all(vt)
    assert [g[0] for g in got] == [(seq0 + i) & M for i in kept] and all(g[5] == 0 for g in got)
    ovr = [i for i in kept if i < lap]
    assert [g[1] == vtile.OVERRUN for g in got] == [i in ovr for i in kept]
    rest = [i for i in kept if i >= lap]
    want_res, want_m, want_recs, want_tags = ref.run([frags[i] for i in rest], depth, seed)
    gr = [g for g in got if g[1] != vtile.OVERRUN]
    assert [g[1] for g in gr] == want_res
    assert vt.metrics() == want_m and vt.overruns() == len(ovr)
    for k, (seqv, r, chunk, sz, tag, _) in enumerate(gr):
        if r == vtile.PUBLISH:
            assert _same_record(vt.record(chunk, sz), want_recs[k], len(frags[rest[k]][0])), k
            assert tag == want_tags[k]
    assert sum(1 for r in want_res if r == vtile.PUBLISH) > 20
    vt.close()
    L.fdgpu_mcache_delete(mc)
    engine.host_unregister(buf)


def test_vtile_gossip_vote_past_frame():
    """The gossip tile publishes every vote update as a 1297-byte frame (FD_GOSSIP_UPDATE_SZ_VOTE,
    fd_gossip_private.h:80), which holds 1225 bytes of vote.txn; the reference tile copies vote.txn_sz
    bytes regardless (fd_verify_tile.c:91-95).  A 1232-byte vote transaction in such a frame -- its last
    7 bytes past the frame, where the update message's vote.txn array continues in the link's dcache --
    verifies and publishes whole through the stem's chunk path, as in the reference; a txn_sz past the
    1232-byte array is corrupt (-4).  Given by pointer (only the frame's bytes known readable), the same
    frame is refused (-4) without reading past it (a short frame must not be over-read)."""
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(4, synth.LARGE_NOOP, seed=9)
    txns = [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    assert all(len(t) == 1232 for t in txns)
    vt = vtile.VTile(device=0, batch_txn=64, tcache_depth=1024)
    # the gossip link's dcache: one 2048-byte frame slot (32 chunks) per frag, room for an MTU frame past wmark
    region = np.zeros(8 * 2048 + 2048, np.uint8)
    assert vt.set_in(2, vtile.IN_GOSSIP, region.ctypes.data, 0, 7 * 32) == 0
    for i, t in enumerate(txns):
        msg = np.frombuffer(vtile.gossip_vote_msg(t), np.uint8)      # 72 + 1232 = 1304 bytes of message
        assert len(msg) == 1304
        region[i * 2048: i * 2048 + 1304] = msg
        assert vt.during_frag_chunk(2, i, vtile.GOSSIP_TAG_VOTE, i * 32, vtile.GOSSIP_MSG_SZ) == 0
    bad = region[:2048].copy()
    region[5 * 2048: 6 * 2048] = bad
    region[5 * 2048 + 64: 5 * 2048 + 72] = np.frombuffer(np.uint64(1233).tobytes(), np.uint8)
    assert vt.during_frag_chunk(2, 9, vtile.GOSSIP_TAG_VOTE, 5 * 32, vtile.GOSSIP_MSG_SZ) == -4
    # by pointer: a short frame (the 1297-byte frame alone, nothing readable after it) claiming 1232 bytes
    short = np.frombuffer(bad[:vtile.GOSSIP_MSG_SZ].tobytes(), np.uint8).copy()
    assert vt.during_frag_at(short.ctypes.data, vtile.GOSSIP_MSG_SZ, 10, in_idx=2) == -4
    # ... and a frame that holds its whole vote transaction is taken
    whole = np.frombuffer(bytes(bad[:1304]), np.uint8).copy()
    got = _drain_all(vt)
    assert [g[1] for g in got] == [vtile.PUBLISH] * 4 and [g[5] for g in got] == [2] * 4
    for (seq, r, chunk, sz, tag, _), t in zip(got, txns):
        rec = vt.record(chunk, sz)
        assert rec[80:80 + 1232] == t and rec[8:10] == (1232).to_bytes(2, "little")
    assert vt.during_frag_at(whole.ctypes.data, 1304, 11, in_idx=2) == 0
    got = _drain_all(vt)
    assert [g[1] for g in got] == [vtile.DEDUP_FAIL]          # (txns[0] again: an HA duplicate)
    vt.close()


def _same_record(rec, want, payload_sz):
    """published records agree but for the alignment pad byte between payload and fd_txn_t"""
    hl = 80 + payload_sz
    return len(rec) == len(want) and rec[:hl] == want[:hl] and rec[(hl + 1) & ~1:] == want[(hl + 1) & ~1:]


def _run_frags(vt, frags, seq0=0):
    from firedancer_amd import vtile
    out = []
    for i, (p, b) in enumerate(frags):
        while vt.during_frag(vtile.frag_bytes(p, b), seq0 + i) == -2:
            out += vt.after_frags(blocking=True)
    vt.flush()
    while vt.pending():
        out += vt.after_frags(blocking=True)
    return [r for _, r, _, _, _, _ in out]


def test_reference_tile_scenarios():
    """The four fd_txn_verify scenarios of src/disco/verify/test_verify.c:161-347 on its own real
    transactions, through the GPU tile.  dedup=0 calls are bundle frags (each its own bundle id);
    fd_tcache_reset is a fresh tile."""
    import json
    from firedancer_amd import vtile
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "verify_tile_txns.json")))
    V1, V2 = bytes.fromhex(d["valid_txn_1sig"]), bytes.fromhex(d["valid_txn_2sigs"])
    I1, I2 = bytes.fromhex(d["invalid_txn_same_1sig"]), bytes.fromhex(d["invalid_txn_2sigs"])
    I64 = bytes.fromhex(d["invalid_txn_1sig_same_64bit"])
    P, F, D = vtile.PUBLISH, vtile.VERIFY_FAIL, vtile.DEDUP_FAIL

    def tile():
        return vtile.VTile(device=0, batch_txn=64, tcache_depth=128)

    # test_verify_success (:161-208)
    assert _run_frags(tile(), [(V2, 0), (V2, 0), (V2, 0), (V2, 1), (V1, 0), (V1, 0), (V1, 0)]) == [P, D, D, P, P, D, D]
    # test_verify_invalid_sigs_success (:210-237): no dedup for failed txns
    assert _run_frags(tile(), [(I2, 0), (I2, 0)]) == [F, F]
    # test_verify_invalid_dedup_success (:239-311)
    assert _run_frags(tile(), [(I1, 0), (V1, 0)]) == [F, P]
    assert _run_frags(tile(), [(V1, 0), (I1, 0)]) == [P, D]
    assert _run_frags(tile(), [(V1, 2), (I1, 3), (I1, 0), (I1, 0)]) == [P, F, F, F]
    # test_verify_invalid_dedup_with_collision_success (:313-347)
    assert _run_frags(tile(), [(V1, 0), (I64, 0)]) == [P, F]


@pytest.mark.parametrize("zero_copy", [False, True])
def test_stream_bench_small(zero_copy):
    """The configs[4] harness end to end at a small size: every frag gets a verdict (with and
    without zero-copy intake)."""
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(4096, synth.LARGE_NOOP, seed=9)
    st = vtile.stream_bench(payload, desc["payload_off"], desc["payload_sz"], n_frags=50000, tiles=2, batch_txn=1024,
                            mcache_depth=8192, zero_copy=zero_copy)
    assert st["frags"] == 50000 and st["overruns"] == 0
    m = st["metrics"]
    # 4096 distinct payloads cycled: the first copy of each publishes per tile, repeats are HA duplicates
    assert m[0] == 0 and m[1] == 0 and m[4] + m[2] == 50000 and m[4] >= 4096
    assert st["lat_p99_us"] > 0


@pytest.mark.parametrize("tiles,reliable,zero_copy,producers", [(3, True, True, 1), (1, True, True, 1), (2, True, False, 1),
                                                           (4, False, True, 1), (3, True, True, 2), (2, False, True, 3)])
def test_stream_run_link(tiles, reliable, zero_copy, producers):
    """The configs[4] link (fdgpu_stream_run): Q producer links, every tile reads every link and takes
    seq % T == i of each, polling its own lines only.  Reliable: every frag gets exactly one verdict and the signature count is that of the
    frags' payloads; unreliable: verdicts + frags lost to overruns = frags published."""
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(3000, synth.MULTI, seed=21)
    n = 40000 + tiles                                   # not a multiple of T: ragged last round
    st = vtile.stream_run(payload, desc["payload_off"], desc["payload_sz"], n_frags=n, tiles=tiles, batch_txn=2048,
                          mcache_depth=16384 if reliable else 4096, zero_copy=zero_copy, reliable=reliable,
                          producers=producers)
    assert st["frags"] == n
    assert st["verdicts"] + st["lost"] == n
    sig_cnt = np.array([payload[o] for o in desc["payload_off"]], np.uint64)
    if reliable:
        assert st["lost"] == 0 and st["verdicts"] == n and st["overruns"] == 0
        # producer q of Q publishes n_q frags, frag s -> payload (s Q + q) % n_payload
        nq = [n // producers + (q < n % producers) for q in range(producers)]
        idx = np.concatenate([(np.arange(nq[q]) * producers + q) % len(desc) for q in range(producers)])
        assert st["sigs"] == int(sig_cnt[idx].sum())
        m = st["metrics"]
        assert m[0] == 0 and m[1] == 0 and sum(m) == n          # no parse / verify failures in valid txns
    else:
        assert st["verdicts"] > 0


@pytest.mark.parametrize("nctx,reliable,rate,split,excl", [(2, True, 0.0, 1, -1), (3, True, 0.0, 1, -1), (2, False, 2e6, 1, -1),
                                                       (2, True, 0.0, 0, 1), (2, False, 2e6, 0, 0), (3, False, 2e6, 1, 1),
                                                       (2, False, 2e6, 0, -1)])
def test_stream_run_cu_split(nctx, reliable, rate, split, excl):
    """Each engine context of a tile on its own share of the CUs the gathers leave (fdgpu_vtile_opts_t.cu_split,
    fdgpu_ed25519_reserve_cus) and / or its latency-path workgroups alone on their CUs (cu_exclusive,
    fdgpu_ed25519_set_cu_exclusive): every frag still gets one verdict, all published, signatures counted."""
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(3000, synth.MULTI, seed=23)
    n = 30001
    st = vtile.stream_run(payload, desc["payload_off"], desc["payload_sz"], n_frags=n, tiles=1, batch_txn=2048,
                          mcache_depth=1 << 16, reliable=reliable, rate_fps=rate, nctx=nctx, gather_cus=16, cu_split=split,
                          cu_exclusive=excl)
    assert st["frags"] == n and st["verdicts"] + st["lost"] == n
    assert st["lost"] == 0 and st["verdicts"] == n and st["overruns"] == 0
    m = st["metrics"]
    assert m[0] == 0 and m[1] == 0 and sum(m) == n
    sig_cnt = np.array([payload[o] for o in desc["payload_off"]], np.uint64)
    assert st["sigs"] == int(sig_cnt[np.arange(n) % len(desc)].sum())


@pytest.mark.parametrize("zero_copy", [False, True])
@pytest.mark.parametrize("rr_idx", [0, 1])
def test_vtile_in_kinds_vs_reference(oracle, rr_idx, zero_copy):
    """The reference tile's four in kinds (fd_verify_tile.c:7-10) through the GPU tile, verify:rr_idx of 2:
    QUIC frags and bundle-tile packets round robin, bundles (sig != 0) only on verify:0, gossip updates
    round robin and only votes (whose txn becomes a fresh record, fd_verify_tile.c:85-95), send frags
    always -- interleaved in stem order.  Which frags the tile keeps (before_frag), each kept frag's
    outcome, the metrics, the published records and the HA dedup tags equal the reference tile's
    (oracle/_ref/libfdref_tile.so, ref_tile_run_kinds).  zero_copy: QUIC / bundle / send records stay in
    a registered in dcache (one link per kind); gossip votes are host-built records either way."""
    pytest.importorskip("xxhash")
    from firedancer_amd import engine, vtile
    from oracle.oracle import RefTile
    from kind_stream import make_kind_stream
    try:
        ref = RefTile()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"reference tile build unavailable: {e}")
    frags = make_kind_stream(31)
    depth, seed = 1 << 12, 0x77aa
    want_res, want_m, want_recs, want_tags = ref.run_kinds([(k, g, q, fb) for k, g, q, fb, _, _ in frags], rr_idx, 2,
                                                           depth, seed)
    vt = vtile.VTile(device=0, batch_txn=64, tcache_depth=depth, seed=seed)
    vt.set_round_robin(rr_idx, 2)
    if zero_copy:
        recs = [fb if k != vtile.IN_GOSSIP else b"" for k, _, _, fb, _, _ in frags]
        buf, offs = in_dcache([r if r else bytes(64) for r in recs])
        engine.host_register(buf)
        assert vt.set_in_links([None] * 4) == 0
    for k in range(4):                    # in link k carries kind k (the stem's in_idx, the tile's in_kind[ in_idx ])
        assert vt.set_in(k, k) == 0
    got, kept = [], []
    for i, (k, g, q, fb, _, _) in enumerate(frags):
        if vt.before_frag(k, q, g):
            continue
        kept.append(i)
        while True:
            if zero_copy and k != vtile.IN_GOSSIP:
                rc = vt.during_frag_at(buf.ctypes.data + offs[i], len(fb), q, in_idx=k)
            else:
                rc = vt.during_frag(fb, q, in_idx=k)
            if rc != -2:
                break
            got += vt.after_frags(blocking=True)
        assert rc == 0, rc
        if i % 29 == 0:
            got += vt.after_frags(blocking=False)
    vt.flush()
    while vt.pending():
        got += vt.after_frags(blocking=True)
    assert kept == [i for i, r in enumerate(want_res) if r != -2]
    assert [g[0] for g in got] == [frags[i][2] for i in kept]
    assert [g[5] for g in got] == [frags[i][0] for i in kept]
    assert [g[1] for g in got] == [want_res[i] for i in kept]
    assert vt.metrics() == want_m
    bad = []
    for (seqv, r, chunk, sz, tag, _), i in zip(got, kept):
        if r != vtile.PUBLISH:
            continue
        rec, want = vt.record(chunk, sz), want_recs[i]
        hl = 80 + len(frags[i][4])
        same = len(rec) == len(want) and rec[(hl + 1) & ~1:] == want[(hl + 1) & ~1:] and rec[80:hl] == want[80:hl]
        if frags[i][0] == vtile.IN_GOSSIP:     # a vote record: payload_sz, txn_t_sz, bundle id (the rest is stale there)
            same = same and rec[8:12] == want[8:12] and rec[24:32] == want[24:32]
        else:
            same = same and rec[:80] == want[:80]
        if not same or tag != want_tags[i]:
            bad.append(i)
    assert bad == []
    assert sum(1 for i in kept if frags[i][0] == vtile.IN_GOSSIP and want_res[i] == vtile.PUBLISH) > 5
    vt.close()
    if zero_copy:
        engine.host_unregister(buf)


def test_host_register_shared_counts_references():
    """fdgpu_host_register_shared: the same range taken twice -- two handles on one mcache ring --
    stays mapped until both unregister; another size at the same start is refused; a range an owner registered
    with fdgpu_host_register is never shared (1: nothing taken) and goes at the owner's one unregister."""
    from firedancer_amd import engine
    L = engine.load_library()
    buf = np.zeros(3 * 4096, np.uint8)
    base = buf.ctypes.data
    off = (-base) % 4096                                   # a whole page-aligned range inside buf
    p, n = base + off, 2 * 4096
    vp, ul = ctypes.c_void_p, ctypes.c_ulong
    assert L.fdgpu_host_register_shared(vp(p), ul(n)) == 0
    assert L.fdgpu_host_register_shared(vp(p), ul(n)) == 0
    assert L.fdgpu_host_register_shared(vp(p), ul(4096)) == -2
    assert L.fdgpu_host_register(vp(p), ul(n)) == -2
    assert L.fdgpu_host_dev_ptr(vp(p), n)
    L.fdgpu_host_unregister(vp(p))
    assert L.fdgpu_host_dev_ptr(vp(p), n), "the second reference keeps the range mapped"
    L.fdgpu_host_unregister(vp(p))
    assert not L.fdgpu_host_dev_ptr(vp(p), n)
    assert L.fdgpu_host_register(vp(p), ul(n)) == 0         # an owner's registration
    assert L.fdgpu_host_register_shared(vp(p), ul(n)) == 1
    L.fdgpu_host_unregister(vp(p))
    assert not L.fdgpu_host_dev_ptr(vp(p), n)


def test_two_handles_on_one_mcache_ring():
    """Two tiles' handles wrapping one ring (fdgpu_mcache_wrap): each set_in_links maps the ring's pages once
    more; deleting one handle leaves the other's mapping."""
    from firedancer_amd import vtile
    L = vtile.load()
    depth = 1 << 10
    ring = np.zeros(depth * 32 + 8192, np.uint8)
    lines = ring.ctypes.data + ((-ring.ctypes.data) % 4096) + 256     # an fd_mcache's lines: 256 B into a page
    m1, m2 = L.fdgpu_mcache_wrap(ctypes.c_void_p(lines), depth), L.fdgpu_mcache_wrap(ctypes.c_void_p(lines), depth)
    assert m1 and m2
    v1, v2 = vtile.VTile(device=0, batch_txn=64, tcache_depth=1024), vtile.VTile(device=0, batch_txn=64, tcache_depth=1024)
    try:
        assert v1.set_in_links([m1]) == 0 and v2.set_in_links([m2]) == 0
        from firedancer_amd import engine
        eng = engine.load_library()
        assert eng.fdgpu_host_dev_ptr(ctypes.c_void_p(lines), depth * 32)
        L.fdgpu_mcache_delete(m1)
        assert eng.fdgpu_host_dev_ptr(ctypes.c_void_p(lines), depth * 32), "m2's mapping survives m1's delete"
        L.fdgpu_mcache_delete(m2)
        assert not eng.fdgpu_host_dev_ptr(ctypes.c_void_p(lines), depth * 32)
    finally:
        v1.close(); v2.close()
