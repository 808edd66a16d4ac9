"""CPU: the reference verify tile's per-frag decision (oracle/_ref/libfdref_tile.so -- fd_txn_verify,
the tcache, fd_hash, fd_txn_parse and the AVX-512 verify compiled in place from the reference) on the
frag streams the GPU tile tests use, and on src/disco/verify/test_verify.c's own scenarios.  It is
the expectation of tests/test_gpu_vtile.py; the sequential Python model there must agree with it."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ref_tile():
    from oracle.oracle import RefTile
    try:
        return RefTile()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"reference tile build unavailable: {e}")


@pytest.mark.parametrize("seed,depth", [(11, 32), (11, 1 << 12), (12, 1 << 12)])
def test_model_matches_reference_tile(ref_tile, oracle, seed, depth):
    pytest.importorskip("xxhash")
    from test_gpu_vtile import make_stream, model
    frags = make_stream(seed=seed)
    hseed = 0x1234abcd
    want_res, want_m, want_recs, tags = ref_tile.run(frags, depth, hseed)
    res, m, recs = model(oracle, frags, hseed, depth)
    assert res == want_res and m == want_m
    assert sum(m[:4]) > 100 and m[2] > 10 and m[3] > 0
    # published records: the model's header + fd_txn_t (the pad byte between payload and fd_txn_t
    # is unspecified) equal the reference's
    assert sorted(recs) == sorted(want_recs)
    for i, (head, timg) in recs.items():
        r = want_recs[i]
        assert r[: len(head)] == head and r[(len(head) + 1) & ~1:] == timg


def test_reference_tile_scenarios(ref_tile):
    """src/disco/verify/test_verify.c:161-347 on its own transactions (bundle frags stand for
    dedup=0 calls; fd_tcache_reset is a fresh run)."""
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "verify_tile_txns.json")))
    V1, V2 = bytes.fromhex(d["valid_txn_1sig"]), bytes.fromhex(d["valid_txn_2sigs"])
    I1, I2 = bytes.fromhex(d["invalid_txn_same_1sig"]), bytes.fromhex(d["invalid_txn_2sigs"])
    I64 = bytes.fromhex(d["invalid_txn_1sig_same_64bit"])
    P, F, D = 0, 2, 3

    def run(frags):
        return ref_tile.run(frags, 128, 0x5eed)[0]
    assert run([(V2, 0), (V2, 0), (V2, 0), (V2, 1), (V1, 0), (V1, 0), (V1, 0)]) == [P, D, D, P, P, D, D]
    assert run([(I2, 0), (I2, 0)]) == [F, F]
    assert run([(I1, 0), (V1, 0)]) == [F, P]
    assert run([(V1, 0), (I1, 0)]) == [P, D]
    assert run([(V1, 2), (I1, 3), (I1, 0), (I1, 0)]) == [P, F, F, F]
    assert run([(V1, 0), (I64, 0)]) == [P, F]


def _before_frag_model(rr_idx, rr_cnt, kind, seq, sig):
    """fd_verify_tile.c:36-59, as the harness and the GPU tile restate it"""
    if (kind == 1 and not sig) or kind == 0:
        return seq % rr_cnt != rr_idx
    if kind == 1:
        return rr_idx != 0
    if kind == 2:
        return seq % rr_cnt != rr_idx or sig != 3
    return False


@pytest.mark.parametrize("rr_idx", [0, 1])
def test_reference_tile_in_kinds(ref_tile, oracle, rr_idx):
    """The harness's in-kind dispatch (before_frag + during_frag, fd_verify_tile.c:36-101, restated in
    ref_tile_harness.c over the reference's own fd_gossip_update_message_t) against a model: the frags
    this tile keeps are exactly the model's, and their outcomes are the reference tile's after_frag
    outcomes of the records the model's during_frag builds (gossip votes -> a fresh record of the vote
    txn with bundle id 0)."""
    pytest.importorskip("xxhash")
    from kind_stream import make_kind_stream
    frags = make_kind_stream(31)
    depth, seed = 1 << 12, 0x77aa
    res, m, recs, tags = ref_tile.run_kinds([(k, g, q, fb) for k, g, q, fb, _, _ in frags], rr_idx, 2, depth, seed)
    keep = [i for i, (k, g, q, _, _, _) in enumerate(frags) if not _before_frag_model(rr_idx, 2, k, q, g)]
    assert [i for i, r in enumerate(res) if r != -2] == keep
    kinds = {k for i in keep for k in [frags[i][0]]}
    assert kinds == {0, 1, 2, 3}
    # the kept frags as plain (payload, bundle id) records through the single-kind reference run
    want_res, want_m, _, _ = ref_tile.run([(frags[i][4], frags[i][5]) for i in keep], depth, seed)
    assert [res[i] for i in keep] == want_res and m == want_m
    assert sum(m[:4]) > 20
