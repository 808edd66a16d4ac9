"""GPU: INTEGRATION.md section 2's tile patch inside the reference's own stem run loop publishes the same stream as
the reference tile (VERDICT r04 Missing 2).

oracle/_ref/libfdref_stem.so runs src/disco/stem/fd_stem.c's STEM_(run1) (compiled in place) with the GPU tile's
callbacks over reference tango objects: a producer thread publishing fd_txn_m_t records on an fd_mcache / dcache
in link (unreliable, as quic_verify), the stem's in fseq and metrics, and an out fd_mcache whose reliable
consumer (a stand-in for the dedup tile, verify_dedup being reliable) returns credits through an fd_fseq.  The
run exercises the stem's credit callbacks (launch / drain / publish in BEFORE_CREDIT / AFTER_CREDIT, at most
STEM_BURST publishes when the out link has the credits), RETURNABLE_FRAG (frags the tile could not take yet are
handed back), downstream backpressure, and, with a lapping producer, the stem's own overrun handling.

Per frag: the tile's verdict equals the reference tile's (oracle/_ref/libfdref_tile.so, the same frags in the
same order), and the consumer receives exactly the reference's published records, in order (XXH64 of each
fd_txn_m_t record as read from the out link, the alignment byte before the fd_txn_t zeroed on both sides)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_stream_parity import payload_set, _with_hs_top  # noqa: E402

pytestmark = pytest.mark.gpu

DEPTH, SEED = 1 << 16, 0x5EED
OVERRUN = 5


@pytest.fixture(scope="module")
def stem():
    from oracle.oracle import RefStem
    try:
        return RefStem()
    except FileNotFoundError as e:
        pytest.skip(f"stem harness not built: {e}")


@pytest.fixture(scope="module")
def ref():
    from oracle.oracle import RefTile
    try:
        return RefTile()
    except (FileNotFoundError, RuntimeError) as e:
        pytest.skip(f"reference tile build unavailable: {e}")


@pytest.fixture(scope="module")
def pays():
    return _with_hs_top(payload_set())


def _rec_hash(r: bytes, payload_sz: int) -> int:
    import xxhash
    r = bytearray(r)
    pe = 80 + payload_sz
    if pe & 1 and pe < len(r):
        r[pe] = 0
    return xxhash.xxh64(bytes(r), seed=0).intdigest()


def _check(ref, pays, st, tr, cons):
    assert st["rc"] == 0 and st["err"] == 0, st
    seq, res, tag = tr
    assert st["verdicts"] == len(seq) == st["traced"]
    assert np.all(np.diff(seq.astype(np.int64)) > 0), "verdicts out of frag order"
    keep = res != OVERRUN
    kseq, kres, ktag = seq[keep], res[keep].astype(int), tag[keep]
    n = len(pays)
    frags = [(pays[int(s) % n], 0) for s in kseq]
    want, metrics, recs, tags = ref.run(frags, DEPTH, SEED)
    bad = np.nonzero(kres != np.array(want))[0]
    assert len(bad) == 0, f"{len(bad)} outcomes differ, first {bad[:5]}: gpu {kres[bad[:5]]} ref {np.array(want)[bad[:5]]}"
    pub = [i for i, r in enumerate(want) if r == 0]
    assert [int(ktag[i]) for i in pub] == [tags[i] for i in pub], "dedup tags"
    # the consumer got exactly the reference's published records, in order, through the stem's out link
    c_hash, c_sz = cons
    assert st["published"] == len(pub) == st["consumed"] == len(c_hash), (st, len(pub))
    want_h = [_rec_hash(recs[i], len(frags[i][0])) for i in pub]
    assert [int(x) for x in c_sz] == [len(recs[i]) for i in pub], "record sizes"
    mism = [j for j in range(len(pub)) if int(c_hash[j]) != want_h[j]]
    assert mism == [], f"{len(mism)} published records differ, first {mism[:5]}"
    assert st["tile_metrics"][:4] == metrics[:4]
    return len(kseq)


@pytest.mark.parametrize("zero_copy", [False, True])
def test_stem_publishes_the_reference_stream(stem, ref, pays, zero_copy):
    """No lapping (in link deeper than the run): every frag reaches the tile once; the consumer receives the
    reference tile's published stream.  Host-copy intake is the reference's own during_frag; zero-copy intake
    lets the GPU copy from the registered in dcache."""
    n = 60_000
    st, tr, cons = stem.run(pays, n, in_depth=1 << 17, out_depth=1024, batch_txn=1024, zero_copy=zero_copy)
    assert st["taken"] == n and st["filtered"] == 0 and st["link_consumed"] == n
    assert st["link_overrun_polling_frags"] == 0 and st["link_overrun_reading_frags"] == 0
    assert _check(ref, pays, st, tr, cons) == n


def test_stem_backpressure_and_returned_frags(stem, ref, pays):
    """A slow downstream consumer (a 200 us pause every 256 frags on a 128-deep out link) backpressures the stem
    (its BACKPRESSURE_COUNT metric); small GPU batches fill the tile's staging, so during_frag hands frags back
    (RETURNABLE_FRAG) and the stem polls them again -- nothing is lost or reordered."""
    n = 40_000
    st, tr, cons = stem.run(pays, n, in_depth=1 << 17, out_depth=128, batch_txn=128, consumer_pause_every=256,
                            consumer_pause_ns=200_000)
    assert st["backpressure_count"] > 0, st
    assert st["returned"] > 0, st
    assert st["taken"] == n and st["link_consumed"] == n
    assert _check(ref, pays, st, tr, cons) == n


@pytest.mark.parametrize("zero_copy", [False, True])
def test_stem_lapping_producer(stem, ref, pays, zero_copy):
    """An unthrottled producer laps a 1024-line in link: the stem loses frags at the poll (its overrun metrics)
    and may find a frag overwritten after during_frag took it, which the tile then never publishes.  The frags
    the tile did verify are decided and published exactly as the reference decides the same sequence."""
    n = 200_000
    st, tr, cons = stem.run(pays, n, in_depth=1 << 10, out_depth=1024, batch_txn=1024, zero_copy=zero_copy)
    assert st["link_overrun_polling_frags"] + st["link_overrun_reading_frags"] > 0, "the producer never lapped"
    assert st["taken"] + st["stem_overruns"] <= n
    _check(ref, pays, st, tr, cons)
