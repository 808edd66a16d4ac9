"""GPU edge cases of the boundary: empty batches, odd batch sizes around the
wave / workgroup widths, all-rejected batches (no lane reaches the DSM),
the largest message the drop-in takes, and its documented limit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fa():
    import firedancer_amd
    firedancer_amd.load_library()
    return firedancer_amd


def _keys(oracle, n, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        prv = rng.bytes(32)
        out.append((prv, oracle.public_from_private(prv)))
    return out


def test_empty_batches(fa):
    from firedancer_amd import engine
    eng = fa.Engine(device=0, max_txn=16, max_sig=16, max_payload=4096)
    t, s = eng.verify_txns_host(np.zeros(64, np.uint8), np.zeros(0, engine.DESC_DTYPE))
    assert len(t) == 0 and len(s) == 0
    c, fp, _ = eng.verify_raw_host(np.zeros(64, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint16))
    assert len(c) == 0
    assert len(eng.verify_many([], [], [])) == 0
    eng.flush()
    assert len(eng.poll(16, blocking=True)[0]) == 0
    eng.close()
    assert engine.sha512_batch([]) == []


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 257, 1031])
def test_odd_batch_sizes(fa, oracle, n):
    """Lanes past the end of a wave / workgroup never leak into results."""
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(n, synth.MULTI, max_signers=3, invalid_frac=0.3, seed=n)
    eng = fa.Engine(device=0, max_txn=n, max_sig=nsig, max_payload=payload.nbytes)
    t, s = eng.verify_txns_host(payload, desc)
    eng.close()
    np.testing.assert_array_equal(t, expect)
    ot, os_ = oracle.verify_txns(payload, desc, nsig)
    np.testing.assert_array_equal(s, os_)


def test_all_rejected_before_dsm(fa, oracle):
    """Every signature fails the S < l check: no lane reaches the hash / table / DSM stages."""
    l_le = (2**252 + 27742317777372353535851937790883648493).to_bytes(32, "little")
    msgs, sigs, pubs = [], [], []
    for i, (prv, pub) in enumerate(_keys(oracle, 300)):
        m = bytes([i & 255]) * (i % 200)
        sig = oracle.sign(m, pub, prv)
        msgs.append(m); sigs.append(sig[:32] + l_le); pubs.append(pub)
    eng = fa.Engine(device=0, max_txn=128, max_sig=128, max_payload=128 * 400)
    got = eng.verify_many(msgs, sigs, pubs)
    eng.close()
    assert (got == -1).all()


def test_largest_dropin_message(fa, oracle):
    """fd_ed25519_verify on a 65439-byte message (the 16-bit descriptor limit less 96 bytes of
    signature and key), and one byte more: past the descriptor range the digests come from the batch
    SHA-512 kernel first, and the codes stay the reference's (fd_ed25519_gpu.h)."""
    (prv, pub), = _keys(oracle, 1, seed=11)
    rng = np.random.default_rng(2)
    m = rng.bytes(65439)
    sig = oracle.sign(m, pub, prv)
    assert oracle.verify(m, sig, pub) == 0
    assert fa.fd_ed25519_verify(m, sig, pub) == 0
    bad = bytearray(m); bad[40000] ^= 1
    assert fa.fd_ed25519_verify(bytes(bad), sig, pub) == -3
    m2 = m + b"\0"
    s2 = oracle.sign(m2, pub, prv)
    assert fa.fd_ed25519_verify(m2, s2, pub) == 0 == oracle.verify(m2, s2, pub)
    assert fa.fd_ed25519_verify(m2, sig, pub) == -3 == oracle.verify(m2, sig, pub)


@pytest.mark.parametrize("frac", [1.0, 0.5])
def test_r_check_slow_path(fa, oracle, frac):
    """Signatures whose R does not match [k](-A)+[S]B take the deferred full
    decode of R (fd_rslow_kernel, compacted across blocks): every one of
    them, or every other one, in a 5000-signature batch."""
    from firedancer_amd import synth
    n = 5000
    payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=31)
    rng = np.random.default_rng(5)
    bad = rng.choice(n, int(n * frac), replace=False)
    for t in bad:
        payload[int(desc["payload_off"][t]) + 700] ^= 0x10      # message byte -> ERR_MSG
    eng = fa.Engine(device=0, max_txn=n, max_sig=nsig, max_payload=payload.nbytes)
    t, s = eng.verify_txns_host(payload, desc)
    eng.close()
    want = np.zeros(n, np.int8); want[bad] = -3
    np.testing.assert_array_equal(t, want)
    ot, os_ = oracle.verify_txns(payload, desc, nsig, threads=16)
    np.testing.assert_array_equal(t, ot)


@pytest.mark.parametrize("every,ntx", [(1, 3000), (3, 3000), (50, 200000), (97, 300000)])
def test_half_size_slow_list(fa, oracle, every, ntx):
    """Half-size path: signatures without a short (c0, c1) take the full 253-bit walk off a compacted
    list (the head in fd_dsmh_kernel's first blocks, the rest in fd_dsm_slow_kernel).  Forced here for
    every / every 3rd / 50th / 97th signature (fdgpu_debug_opts_t.half_force_slow) in adversarial multi-signer
    batches: codes equal the oracle's.  At 2 % (every 50th of ~500K signatures) the list overflows the
    head into fd_dsm_slow_kernel, and a slow signature's code is final long before the last
    half-size blocks start (they must not take it for a half-size one)."""
    from firedancer_amd import synth
    from firedancer_amd import engine
    payload, desc, expect, nsig = synth.make_batch(ntx, synth.MULTI, max_signers=4, invalid_frac=0.3, seed=77 + every,
                                                   threads=16)
    engine.debug_set_opts(half=1, small_batch_max=0, half_force_slow=every)
    try:
        eng = fa.Engine(device=0, max_txn=len(desc), max_sig=nsig, max_payload=payload.nbytes)
    finally:
        engine.debug_reset_opts()
    t, s = eng.verify_txns_host(payload, desc)
    eng.close()
    np.testing.assert_array_equal(t, expect)
    ot, os_ = oracle.verify_txns(payload, desc, nsig, threads=16)
    np.testing.assert_array_equal(s, os_)


@pytest.mark.parametrize("every", [1, 5])
def test_half_size_slow_list_engine_paths(fa, oracle, engine_path, every):
    """The forced slow list on every engine path at a latency-path batch size (~6K signatures): the 8-, 4-
    and 2-lane walk kernels verify the list at their end (slowl_tail), the one-lane walk in
    fd_dsm_slowl_kernel, the throughput path in fd_dsmh_kernel's head blocks.  Every signature (1) or every
    5th, in adversarial multi-signer batches: codes equal the oracle's, and the list holds the forced
    signatures that passed the S check."""
    from conftest import engine_opts
    from firedancer_amd import engine, synth
    payload, desc, expect, nsig = synth.make_batch(2500, synth.MULTI, max_signers=4, invalid_frac=0.3,
                                                   seed=131 + every, threads=16)
    assert nsig <= 8192                                 # every lane count's batch limit (FD_DSM8_MAX)
    engine.debug_set_opts(**engine_opts(engine_path, half_force_slow=every))
    try:
        eng = fa.Engine(device=0, max_txn=len(desc), max_sig=nsig, max_payload=payload.nbytes)
    finally:
        engine.debug_set_opts(**engine_opts(engine_path))
    try:
        t, s = eng.verify_txns_host(payload, desc)
        if engine_path != "throughput_full":        # (a signature whose S check fails never reaches the list)
            assert (nsig + every - 1) // every // 2 < eng.slow_count() <= (nsig + every - 1) // every
    finally:
        eng.close()
    np.testing.assert_array_equal(t, expect)
    ot, os_ = oracle.verify_txns(payload, desc, nsig, threads=16)
    np.testing.assert_array_equal(s, os_)


@pytest.mark.parametrize("path", ["throughput", "latency"])
def test_half_size_no_silent_fallback(fa, path):
    """Hash-distributed k always has a short (c0, c1) within 2^159: a valid batch takes the half-size walk
    for every signature (slow list empty).  A device reduction that failed its own congruence check would
    still verify correctly through the full walk -- only this count shows it.  The forced slow list counts
    exactly the forced signatures."""
    from firedancer_amd import engine, synth
    sbm = 0 if path == "throughput" else 2**63
    payload, desc, expect, nsig = synth.make_batch(20000, synth.MULTI, max_signers=3, invalid_frac=0.0, seed=91,
                                                   threads=16)
    engine.debug_set_opts(half=1, small_batch_max=sbm)
    try:
        eng = fa.Engine(device=0, max_txn=len(desc), max_sig=nsig, max_payload=payload.nbytes)
    finally:
        engine.debug_reset_opts()
    t, _ = eng.verify_txns_host(payload, desc)
    assert eng.slow_count() == 0
    eng.close()
    np.testing.assert_array_equal(t, expect)
    engine.debug_set_opts(half=1, small_batch_max=sbm, half_force_slow=7)
    try:
        eng = fa.Engine(device=0, max_txn=len(desc), max_sig=nsig, max_payload=payload.nbytes)
    finally:
        engine.debug_reset_opts()
    t, _ = eng.verify_txns_host(payload, desc)
    assert eng.slow_count() == (nsig + 6) // 7
    eng.close()
    np.testing.assert_array_equal(t, expect)


def test_message_lengths_at_sha512_block_edges(fa, oracle, engine_path):
    """k = SHA-512(R || A || M) for inputs that end exactly at, just before and just after a 128-byte block
    boundary, and where the 0x80 byte and the 16-byte length do or do not fit the last data block
    (64 + msg_sz mod 128 around 0, 111 and 112): the full-block fast path of fd_sha512_RAM must give the
    same codes as the oracle -- valid signatures verify, a flipped message bit gives ERR_MSG."""
    sizes = sorted({max(0, L - 64) for b in range(0, 11) for d in (-1, 0, 1, 111, 112, 113)
                    for L in (128 * b + d,) if L >= 64} | {0, 1, 2})
    keys = _keys(oracle, len(sizes), seed=11)
    rng = np.random.default_rng(12)
    msgs, sigs, pubs, want = [], [], [], []
    for (prv, pub), n in zip(keys, sizes):
        m = rng.bytes(n)
        sig = oracle.sign(m, pub, prv)
        msgs.append(m); sigs.append(sig); pubs.append(pub); want.append(0)
        if n:
            f = bytearray(m); f[n // 2] ^= 1
            msgs.append(bytes(f)); sigs.append(sig); pubs.append(pub); want.append(-3)
    eng = fa.Engine(device=0, max_txn=len(msgs), max_sig=len(msgs), max_payload=len(msgs) * 1600 + 4096)
    got = eng.verify_many(msgs, sigs, pubs)
    eng.close()
    np.testing.assert_array_equal(np.asarray(got), np.asarray(want))
