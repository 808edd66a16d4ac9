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
