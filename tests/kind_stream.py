"""A verify tile's mixed input (test data): frags of all four in kinds of src/disco/verify/fd_verify_tile.c:7-10
-- QUIC, bundle (packets with sig 0 and bundles with sig != 0), gossip updates (votes and other tags) and send
-- interleaved in stem order, each with its own link's seq.  Payloads come from the GPU tile tests' stream
(valid, invalid, unparsable, HA duplicates, bundles with failing members)."""
import numpy as np

from test_gpu_vtile import make_stream

IN_QUIC, IN_BUNDLE, IN_GOSSIP, IN_SEND = range(4)
GOSSIP_TAG_VOTE = 3


def gossip_msg(txn: bytes, tag: int) -> bytes:
    from firedancer_amd import vtile
    return vtile.gossip_vote_msg(txn, tag=tag)


def make_kind_stream(seed: int = 31):
    """[(in_kind, sig, seq, frag bytes, payload, bundle_id)] in stem order."""
    from firedancer_amd import vtile
    rng = np.random.default_rng(seed)
    base = make_stream(seed=seed)
    seqs = [0, 0, 0, 0]
    out = []

    def emit(kind, sig, fb, payload, bid):
        out.append((kind, sig, seqs[kind], fb, payload, bid))
        seqs[kind] += 1

    i = 0
    while i < len(base):
        p, bid = base[i]
        if bid:                                     # a bundle: all its members, from the bundle link (sig != 0)
            j = i
            while j < len(base) and base[j][1] == bid:
                emit(IN_BUNDLE, 1 + (bid % 7), vtile.frag_bytes(base[j][0], bid), base[j][0], bid)
                j += 1
                if rng.random() < 0.3:              # QUIC frags arrive between a bundle's members
                    q = base[int(rng.integers(len(base)))][0]
                    emit(IN_QUIC, 0, vtile.frag_bytes(q, 0), q, 0)
            i = j
            continue
        r = rng.random()
        if r < 0.55:
            emit(IN_QUIC, 0, vtile.frag_bytes(p, 0), p, 0)
        elif r < 0.70:                              # a bundle-tile packet: a plain txn, round robin
            emit(IN_BUNDLE, 0, vtile.frag_bytes(p, 0), p, 0)
        elif r < 0.88:                              # gossip: mostly votes, some other updates (skipped)
            tag = GOSSIP_TAG_VOTE if rng.random() < 0.75 else int(rng.choice([0, 1, 2, 4, 5]))
            emit(IN_GOSSIP, tag, gossip_msg(p, tag), p, 0)
        else:
            emit(IN_SEND, 0, vtile.frag_bytes(p, 0), p, 0)
        i += 1
    return out
