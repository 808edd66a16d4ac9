"""GPU: the configs[4] stream at scale, frag for frag against the reference tile.

200,000 frags go through the link (fdgpu_link_*: one producer mcache over the in dcache, two verify
tiles with the reference's seq % T round robin, zero-copy intake, one GPU), once over a reliable link
and once over an unreliable one whose unthrottled producer laps a 4096-line mcache, so that tiles lose
frags at the poll and may lose some at the copy.  Every tile records its verdicts in after_frags order
(fdgpu_link_set_trace).  The frags a tile accepted -- every verdict but FDGPU_VTILE_OVERRUN, which the
reference's stem skips before after_frag (src/disco/stem/fd_stem.c:667-686) -- are then run, in the same
order, through the reference tile compiled in place (oracle/_ref/libfdref_tile.so: fd_txn_parse,
fd_txn_verify with its tcache and fd_hash, the AVX-512 verify, after_frag's bundle bookkeeping) with
that tile's dedup seed and depth.  Per frag: the same outcome; for a published frag the same HA dedup
tag and the same fd_txn_m_t record (XXH64 of the record as published in the tile's out dcache, the
alignment byte before the fd_txn_t zeroed on both sides).

The payloads mix valid single-signer 1232-byte transactions, invalid signatures, multi-signer and
200-byte-message transactions, builder transactions and mutations (parse failures), 44K of them, so
the 200K frags repeat each about 4.5 times: tile i always gets the same payloads (seq % 2 == i and the
payload index is seq % n with n even), 22K own frags apart, within the 65,536-deep tcache -- repeats
are HA duplicates."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import txn_builder as tb  # noqa: E402

pytestmark = pytest.mark.gpu

N_FRAGS = 200_000
TILES = 2
DEPTH = 1 << 16          # the link tiles' tcache depth (fd_verify_gpu.c link_tile)
SEED0 = 0x5EED           # link tile i's dedup seed is SEED0 + i


def payload_set():
    from firedancer_amd import synth
    rng = np.random.default_rng(77)
    pays = []
    for kind, ms, inv, n, s in ((synth.LARGE_NOOP, 1, 0.05, 40000, 31), (synth.MULTI, 12, 0.2, 2000, 32),
                                (synth.SMALL_MSG, 1, 0.1, 1200, 33)):
        payload, desc, _, _ = synth.make_batch(n, kind, ms, inv, seed=s)
        pays += [payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes() for d in desc]
    built = [tb.build_txn(rng) for _ in range(400)]
    pays += built + [tb.mutate(rng, built[int(rng.integers(len(built)))]) for _ in range(400)]
    pays = [p for p in pays if 0 < len(p) <= 1232]
    pays = pays[: len(pays) & ~1]                     # even count: a payload always lands on the same tile
    order = rng.permutation(len(pays))
    return [pays[i] for i in order]


def run_leg(pays, reliable, depth, n_frags=N_FRAGS, tiles=TILES, **kw):
    from firedancer_amd import vtile
    sz = np.array([len(p) for p in pays], np.uint16)
    off = np.zeros(len(pays), np.uint32)
    off[1:] = np.cumsum(sz[:-1].astype(np.int64))
    arena = np.frombuffer(b"".join(pays) + bytes(64), np.uint8)
    cfg = dict(batch_txn=8192, max_inflight=2, rate_fps=0.0, nctx=1)
    cfg.update(kw)
    link = vtile.Link(None, create=True, payload=arena, off=off, sz=sz, n_frags=n_frags, tiles=tiles, gpus=1,
                      zero_copy=True, reliable=reliable, mcache_depth=depth, producers=1, **cfg)
    try:
        link.set_trace(n_frags)
        assert link.run(0, 0, True) == 0
        st = link.result(timeout_s=120.0)
        traces = [link.trace(i, n_frags) for i in range(tiles)]
        anomalies = [link.anomalies(i) for i in range(tiles)]
    finally:
        link.close()
    return st, traces, anomalies


def check_tiles(pays, traces, tiles=TILES):
    from firedancer_amd import vtile
    from oracle.oracle import RefTile
    import xxhash
    try:
        ref = RefTile()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"reference tile build unavailable: {e}")
    n = len(pays)
    for i, tr in enumerate(traces):
        keep = tr[tr["result"] != vtile.OVERRUN]
        seqs = keep["seq"]
        assert np.all(keep["in_idx"] == 0), "one producer link: every frag on in link 0"
        assert np.all(seqs % tiles == i), "a tile took a frag of another tile's round-robin share"
        assert np.all(np.diff(seqs.astype(np.int64)) > 0), "verdicts out of frag order"
        frags = [(pays[int(s) % n], 0) for s in seqs]
        res, metrics, recs, tags = ref.run(frags, DEPTH, SEED0 + i)
        got = keep["result"].astype(int)
        bad = np.nonzero(got != np.array(res))[0]
        assert len(bad) == 0, f"tile {i}: {len(bad)} outcomes differ, first at {bad[:5]}: gpu {got[bad[:5]]} ref {np.array(res)[bad[:5]]}"
        pub = np.nonzero(got == vtile.PUBLISH)[0]
        assert len(pub) == len(recs) and len(pub) > 0
        for j in pub:
            r = bytearray(recs[int(j)])
            pe = 80 + len(frags[int(j)][0])
            if pe & 1 and pe < len(r):
                r[pe] = 0
            assert int(keep["rec_sz"][j]) == len(r), f"tile {i} frag {j}: record size"
            assert int(keep["rec_hash"][j]) == xxhash.xxh64(bytes(r), seed=0).intdigest(), f"tile {i} frag {j}: record"
            assert int(keep["tag"][j]) == tags[int(j)], f"tile {i} frag {j}: dedup tag"
        yield i, len(keep), metrics


def test_stream_parity_reliable():
    pays = payload_set()
    st, traces, _ = run_leg(pays, reliable=True, depth=1 << 16)
    assert st["verdicts"] == N_FRAGS and st["lost"] == 0 and st["overruns"] == 0
    assert sum(len(t) for t in traces) == N_FRAGS
    seen = list(check_tiles(pays, traces))
    assert sum(k for _, k, _ in seen) == N_FRAGS
    assert all(m[2] > 0 and m[1] > 0 for _, _, m in seen), "the stream should exercise dedup and verify failures"


def test_stream_parity_unreliable_laps():
    pays = payload_set()
    st, traces, _ = run_leg(pays, reliable=False, depth=1 << 12)
    assert st["verdicts"] + st["lost"] == N_FRAGS
    # the leg must exercise what it is for: tiles lapped at the poll (lost frags), and the verdicts of
    # frags overrun while the GPU copied them recorded as such (the gather-time line re-check)
    assert st["lost"] > 0, "the 4096-line link was never lapped"
    n_ovr = sum(int((t["result"] == 5).sum()) for t in traces)      # FDGPU_VTILE_OVERRUN
    assert n_ovr == st["overruns"]
    assert sum(len(t) for t in traces) == st["verdicts"]
    seen = list(check_tiles(pays, traces))
    assert sum(k for _, k, _ in seen) == st["verdicts"] - st["overruns"]


def _with_hs_top(pays):
    """The payload set plus the eight valid transactions whose half-size scalars are below 2^120
    (tests/golden/hs_top.npz: the inputs that round 4's walks rejected when alone in their wave), each
    spliced in a few times."""
    hs = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "hs_top.npz"))
    special = [hs["txn"][i][: int(hs["payload_sz"][i])].tobytes() for i in range(len(hs["txn"]))]
    out = list(pays)
    for j in range(0, len(out), 997):
        out[j] = special[(j // 997) % len(special)]
    return out


@pytest.mark.parametrize("rate", [2e6, 7.5e6])
def test_stream_parity_paced_latency_two_contexts(rate):
    """The configuration of round 4's withheld valid frag (VERDICT r04 Missing 1): the bench's paced leg --
    one tile, two engine contexts whose batches overlap, the latency path (batches of at most 8,192, 8-lane
    half-size walks), latency-path workgroups alone on their CUs (cu_exclusive, the tile's default), 16 CUs
    reserved for the copies, copies after 25 us -- over an unreliable link deep enough that nothing is
    lapped, at 2M and 7.5M frags/s.  Every frag's verdict, dedup tag and published record equal the
    reference tile's, and no verdict of a valid frag is anything but PUBLISH or a dedup of a repeat."""
    n = 250_000
    pays = _with_hs_top(payload_set())
    st, traces, anomalies = run_leg(pays, reliable=False, depth=1 << 18, n_frags=n, tiles=1, rate_fps=rate,
                                    nctx=2, max_inflight=1, gather_cus=16, copy_wait_ns=25_000, cu_exclusive=0)
    assert st["lost"] == 0 and st["overruns"] == 0 and st["verdicts"] == n, (st["lost"], st["overruns"])
    assert st["batches"] > 0 and st["batch_txns"] / st["batches"] <= 8192
    seen = list(check_tiles(pays, traces, tiles=1))
    assert sum(k for _, k, _ in seen) == n
    # the diagnostics every non-published verdict carries (the payload set holds invalid and unparsable
    # transactions): the GPU batch it came from and the GPU's own code for it
    cnt, first = anomalies[0]
    assert cnt > 0
    for a in first:
        assert a["batch_txns"] > a["batch_pos"] and a["ctx"] < 2 and a["path"] in (8, 4, 2, 1, 0, -1), a
        if a["result"] == 2:                                    # FDGPU_VTILE_VERIFY_FAIL
            assert a["code"] in (-1, -2, -3), a
        elif a["result"] == 1:                                  # FDGPU_VTILE_PARSE_FAIL
            assert a["code"] == -16, a


@pytest.mark.parametrize("rate", [7.5e6])
def test_stream_parity_paced_launch_thread(rate):
    """The paced leg with the tile's launch thread (fdgpu_vtile_opts_t.launcher, the bench's
    --stream-lat-launcher): the tile's thread queues each batch launch and early copy, a thread of its own
    makes the runtime calls.  Frag for frag the same as the reference tile, nothing lost or overrun."""
    n = 250_000
    pays = _with_hs_top(payload_set())
    st, traces, _ = run_leg(pays, reliable=False, depth=1 << 18, n_frags=n, tiles=1, rate_fps=rate, nctx=2,
                            max_inflight=1, gather_cus=16, copy_wait_ns=25_000, cu_exclusive=0, launcher=1)
    assert st["lost"] == 0 and st["overruns"] == 0 and st["verdicts"] == n, (st["lost"], st["overruns"])
    assert st["launcher"][0] >= st["batches"] > 0 and st["launcher"][1] > 0
    seen = list(check_tiles(pays, traces, tiles=1))
    assert sum(k for _, k, _ in seen) == n


def test_stream_parity_reliable_launch_thread():
    """Two reliable max-rate tiles, each with its launch thread: frag for frag the reference tile's."""
    pays = payload_set()
    st, traces, _ = run_leg(pays, reliable=True, depth=1 << 16, launcher=1)
    assert st["verdicts"] == N_FRAGS and st["lost"] == 0 and st["overruns"] == 0
    assert st["launcher"][0] >= st["batches"] > 0
    seen = list(check_tiles(pays, traces))
    assert sum(k for _, k, _ in seen) == N_FRAGS


@pytest.mark.parametrize("reliable", [True, False])
def test_stream_parity_host_copy_threads(reliable):
    """Two tiles whose copy threads write each record into the out dcache while the GPU copy only reads it
    (fdgpu_vtile_opts_t.copy_threads = 2, the bench's --stream-copy-threads): reliable, and unreliable with
    a producer lapping a 4096-line mcache (frags overrun at the poll or found overrun by a copy are never
    published).  Frag for frag the reference tile's verdicts, tags and records."""
    pays = payload_set()
    st, traces, _ = run_leg(pays, reliable=reliable, depth=1 << 16 if reliable else 1 << 12, copy_threads=2)
    if reliable:
        assert st["verdicts"] == N_FRAGS and st["lost"] == 0 and st["overruns"] == 0
    else:
        assert st["verdicts"] + st["lost"] == N_FRAGS and st["lost"] > 0
    assert st["host_copy"][0] == st["verdicts"]          # every frag a tile took was copied by a copy thread
    n_ovr = sum(int((t["result"] == 5).sum()) for t in traces)
    assert n_ovr == st["overruns"]
    seen = list(check_tiles(pays, traces))
    assert sum(k for _, k, _ in seen) == st["verdicts"] - st["overruns"]
