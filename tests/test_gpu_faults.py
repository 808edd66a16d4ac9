"""GPU: the failure edges of the boundary.

* A record larger than a context's payload arena is refused before it is
  staged, in every submit mode (the first record of an empty slot used to
  be accepted at any size and overran the host and device arenas).
* The drop-in fd_ed25519_verify takes messages of any length, as the
  reference does (fd_ed25519_user.c:135-230 has no length limit): beyond
  the 16-bit descriptor range the digests are computed first; codes match
  the oracle.
* The verify tile's fault path: a context whose batch failed never blocks
  after_frags, its frags come back in order as FDGPU_VTILE_GPU_FAULT, the
  other context keeps verifying, and fdgpu_vtile_recover brings it back
  (the reference's failure mode is a loud tile crash, fd_verify_tile.c:74-84).
"""
import ctypes
import os
import sys
import time

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _txn(n=1, seed=5):
    from firedancer_amd import synth
    payload, desc, _, _ = synth.make_batch(n, synth.LARGE_NOOP, seed=seed)
    d = desc[0]
    return payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes(), d


def test_submit_refuses_record_larger_than_arena():
    from firedancer_amd import engine
    L = engine.load_library()
    txn, d = _txn()
    assert len(txn) == 1232
    eng = engine.Engine(device=0, max_txn=64, max_sig=64, max_payload=1024)
    b = np.frombuffer(txn, np.uint8)
    # descriptor and raw copies into the staging slot
    assert L.fdgpu_ed25519_submit(eng.ctx, b.ctypes.data, len(txn), int(d["signature_off"]), int(d["acct_addr_off"]),
                                  int(d["message_off"]), 1, 7) == -4
    assert L.fdgpu_ed25519_submit_raw(eng.ctx, b.ctypes.data, len(txn), 7) == -4
    # in place from a pinned region, and gathered by the GPU
    region = L.fdgpu_host_alloc(1 << 16)
    assert region
    try:
        ctypes.memmove(region + 64, txn, len(txn))
        assert L.fdgpu_ed25519_submit_raw_ref(eng.ctx, region, region + 64, len(txn), 7) == -4
        out = L.fdgpu_host_alloc(1 << 16)
        try:
            assert L.fdgpu_ed25519_submit_raw_gather(eng.ctx, region + 64, out, out + 64, len(txn), 0, len(txn), 7) == -4
        finally:
            L.fdgpu_host_free(out)
    finally:
        L.fdgpu_host_free(region)
    # nothing was queued; a record that fits still goes through
    filling = (ctypes.c_ulong(), ctypes.c_ulong())
    L.fdgpu_ed25519_pipeline_state(eng.ctx, ctypes.byref(filling[0]), ctypes.byref(filling[1]))
    assert filling[0].value == 0 and filling[1].value == 0
    small = txn[:600]
    assert eng.submit_raw(small, 1) == 0
    eng.flush()
    tags, codes, fp, _ = eng.poll_raw(blocking=True)
    assert list(tags) == [1] and codes[0] == engine.FDGPU_ERR_PARSE      # truncated payload: fd_txn_parse rejects it
    eng.close()


@pytest.mark.parametrize("msg_sz", [65535 - 96, 65535 - 95, 70000, 200000])
def test_dropin_long_messages(oracle, msg_sz):
    from firedancer_amd import engine
    rng = np.random.default_rng(msg_sz)
    prv = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pub = oracle.public_from_private(prv)
    msg = rng.integers(0, 256, msg_sz, dtype=np.uint8).tobytes()
    sig = oracle.sign(msg, pub, prv)
    bad_msg = msg[:-1] + bytes([msg[-1] ^ 1])
    bad_s = sig[:32] + b"\xff" * 32
    for m, s in ((msg, sig), (bad_msg, sig), (msg, bad_s)):
        assert engine.fd_ed25519_verify(m, s, pub) == oracle.verify(m, s, pub)
    assert engine.fd_ed25519_verify(msg, sig, pub) == 0
    assert engine.fd_ed25519_verify(bad_msg, sig, pub) == engine.FD_ED25519_ERR_MSG
    # batch over one long message: 3 signers, the second one's signature of another message
    prvs = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(3)]
    pubs = [oracle.public_from_private(p) for p in prvs]
    sigs = [oracle.sign(msg, pk, sk) for pk, sk in zip(pubs, prvs)]
    sigs[1] = oracle.sign(bad_msg, pubs[1], prvs[1])
    got = engine.fd_ed25519_verify_batch_single_msg(msg, b"".join(sigs), b"".join(pubs), 3)
    assert got == oracle.verify_batch_single_msg(msg, b"".join(sigs), b"".join(pubs), 3) == engine.FD_ED25519_ERR_MSG


def test_vtile_fault_path():
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(96, synth.LARGE_NOOP, seed=31)
    frags = [vtile.frag_bytes(payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes()) for d in desc]
    vt = vtile.VTile(device=0, batch_txn=32, tcache_depth=4096, nctx=2)
    # frags 0..31 -> context 0, 32..63 -> context 1 (full batches launch and move the fill on)
    for seq in range(64):
        assert vt.during_frag(frags[seq], seq) == 0
        if seq in (31, 63):
            assert vt.housekeep(3) == 1                # a full batch launches at once and the next context fills
    vt.debug_fault(0)
    assert vt.faulted() == 1
    t0 = time.time()
    got = []
    while vt.pending():
        got += vt.after_frags(blocking=True)
        assert time.time() - t0 < 30, "after_frags spun on a faulted context"
    assert [g[0] for g in got] == list(range(64))
    res = [g[1] for g in got]
    assert res[:32] == [vtile.GPU_FAULT] * 32          # never published, returned in order, no block
    assert res[32:] == [vtile.PUBLISH] * 32            # the healthy context verified its frags
    gm = vt.gpu_metrics()
    assert gm["gpu_fault_frags"] == 32 and gm["faults"] == 1 and gm["batches"] >= 2 and gm["pending"] == 0
    # new frags go to the healthy context while one is faulted; then recover and use both again
    assert vt.during_frag(frags[64], 64) == 0
    vt.flush()
    while vt.pending():
        got += vt.after_frags(blocking=True)
    assert got[-1][1] == vtile.PUBLISH
    assert vt.recover() == 0 and vt.faulted() == 0
    for seq in range(65, 96):
        assert vt.during_frag(frags[seq], seq) == 0
    vt.flush()
    while vt.pending():
        got += vt.after_frags(blocking=True)
    assert [g[1] for g in got[65:]] == [vtile.PUBLISH] * 31
    assert vt.metrics()[4] == 32 + 1 + 31
    vt.close()


def test_vtile_all_contexts_faulted_refuses_intake():
    from firedancer_amd import synth, vtile
    payload, desc, _, _ = synth.make_batch(4, synth.LARGE_NOOP, seed=32)
    frags = [vtile.frag_bytes(payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes()) for d in desc]
    vt = vtile.VTile(device=0, batch_txn=32, tcache_depth=64)
    assert vt.during_frag(frags[0], 0) == 0
    for k in range(3):
        vt.debug_fault(k)
    assert vt.during_frag(frags[1], 1) == -3
    out = vt.after_frags(blocking=True)
    assert [(s, r) for s, r, _, _, _, _ in out] == [(0, vtile.GPU_FAULT)]
    assert vt.recover() == 0
    assert vt.during_frag(frags[1], 1) == 0
    vt.flush()
    out = []
    while vt.pending():
        out += vt.after_frags(blocking=True)
    assert [(s, r) for s, r, _, _, _, _ in out] == [(1, vtile.PUBLISH)]
    vt.close()
