"""GPU: the other batchable callers of SURVEY.md §3 C/D through the C ABI.

* Replay (fd_executor_txn_verify, src/flamenco/runtime/fd_executor.c:1550-1574): every
  transaction of a block, each in its own buffer and already parsed, verified in one
  fdgpu_ed25519_verify_txn_ptrs call; codes equal the oracle's batch verify per transaction.
* Gossip (fd_gossvf_tile.c:360-450): a prune message is accepted if either of its two signable
  forms verifies (:360-371); CRDS values, pings and pongs are independent (msg, sig, pub)
  triples -- fdgpu_ed25519_verify_many_host against the oracle's fd_ed25519_verify.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_replay_block_txn_ptrs(oracle):
    import firedancer_amd as fa
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(3000, synth.MULTI, 12, 0.15, seed=2024)
    payloads = [payload[int(d["payload_off"]): int(d["payload_off"]) + int(d["payload_sz"])].tobytes() for d in desc]
    eng = fa.Engine(device=0, max_txn=1024, max_sig=4096, max_payload=1 << 20)   # several chunks
    got = eng.verify_txn_ptrs(payloads, desc)
    eng.close()
    o_txn, _ = oracle.verify_txns(payload, desc, nsig, threads=16)
    np.testing.assert_array_equal(got, o_txn)
    np.testing.assert_array_equal(got, expect)
    assert (got != 0).sum() > 300


def test_gossip_prune_and_crds(oracle):
    import firedancer_amd as fa
    rng = np.random.default_rng(9)
    msgs, sigs, pubs = [], [], []
    keys = []
    for i in range(64):
        prv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        keys.append((prv, oracle.public_from_private(prv)))
    for i in range(400):
        prv, pub = keys[i % 64]
        m = rng.integers(0, 256, int(rng.integers(0, 1200)), dtype=np.uint8).tobytes()
        s = oracle.sign(m, pub, prv)
        if i % 5 == 1:
            m = m + b"x"                                  # tampered value
        if i % 7 == 3:
            s = s[:32] + bytes(32)                        # zero S: still canonical, equation fails
        msgs.append(m); sigs.append(s); pubs.append(pub)
    # prune: the signature covers the prefixed form for even i, the bare form for odd i
    prefix = b"\xffSOLANA_PRUNE_DATA"
    prune_ok = []
    for i in range(40):
        prv, pub = keys[i]
        body = rng.integers(0, 256, 98 + 32 * (i % 4), dtype=np.uint8).tobytes()
        s = oracle.sign(prefix + body if i % 2 == 0 else body, pub, prv)
        msgs += [prefix + body, body]; sigs += [s, s]; pubs += [pub, pub]
        prune_ok.append(True)
    eng = fa.Engine(device=0, max_txn=256, max_sig=256, max_payload=1 << 18)
    got = eng.verify_many(msgs, sigs, pubs)
    eng.close()
    want = np.array([oracle.verify(m, s, p) for m, s, p in zip(msgs, sigs, pubs)], np.int8)
    np.testing.assert_array_equal(got, want)
    pr = got[400:].reshape(-1, 2)
    assert [bool((pr[i] == 0).any()) for i in range(len(pr))] == prune_ok   # verify_prune's either-form rule
