"""GPU: full-size parity, code for code against the reference.

BASELINE configs[0] (65,536 x 200-byte messages, one device-resident launch),
configs[1] (1,048,576 single-signer 1232-byte txns, all valid),
configs[2] (1,048,576 txns: 10 % injected faults of every synthetic kind --
S >= l, undecodable R / A, small-order R / A, message flip -- plus the
reference's edge encodings (small-order with both sign bits, non-canonical
y = p + k) spliced into R or A of ~1.5 % more) and configs[3] (262,144 txns
of 1..12 signers over one message, 10 % faults), each through the C ABI's
host path (sub-batches of 131,072 with the H2D overlapped, i.e. the
throughput path with the deferred R check and its compacted slow path at
full size), compared transaction by transaction and signature by
signature with the reference's own fd_ed25519_verify_batch_single_msg /
fd_ed25519_verify (oracle/_ref, AVX-512 build; configs[2] also against the
portable build with the engine in portable semantics).  Without the
compiled reference (or an AVX-512 IFMA host) the oracle restatement is the
expectation.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16


def _expectation(variant):
    from oracle.oracle import Oracle, Reference, cpu_has_avx512_ifma
    try:
        if variant == "avx512" and not cpu_has_avx512_ifma():
            raise RuntimeError
        ref = Reference(variant)
        return lambda pay, desc, nsig: ref.verify_txns(pay, desc, nsig, threads=THREADS)
    except (FileNotFoundError, RuntimeError):
        o, sem = Oracle(), (0 if variant == "avx512" else 1)
        return lambda pay, desc, nsig: o.verify_txns(pay, desc, nsig, sem=sem, threads=THREADS)


def _edge_encodings():
    from tests.golden_io import load_vectors
    v = load_vectors()
    e = v["set_id"] == 4
    encs = {bytes(x) for x in v["pub"][e]} | {bytes(x[:32]) for x in v["sig"][e]}
    return np.array([np.frombuffer(x, np.uint8) for x in sorted(encs)])


def _splice_edges(payload, desc, frac, seed):
    """Overwrite R (first signature) or A (first signer's key) of frac of the txns with edge encodings."""
    rng = np.random.default_rng(seed)
    encs = _edge_encodings()
    idx = rng.choice(len(desc), int(frac * len(desc)), replace=False)
    which = rng.integers(0, 2, len(idx))
    pick = rng.integers(0, len(encs), len(idx))
    for t, w, k in zip(idx, which, pick):
        d = desc[t]
        at = int(d["payload_off"]) + (int(d["signature_off"]) if w == 0 else int(d["acct_addr_off"]))
        payload[at: at + 32] = encs[k]
    return len(idx)


def _run(payload, desc, nsig, sem):
    import firedancer_amd as fa
    eng = fa.Engine(device=0, max_txn=len(desc), max_sig=nsig, max_payload=payload.nbytes, semantics=sem)
    try:
        return eng.verify_txns_host(payload, desc)
    finally:
        eng.close()


def _check(got_txn, got_sig, want_txn, want_sig):
    bad = np.nonzero(got_txn != want_txn)[0]
    assert len(bad) == 0, [(int(i), int(got_txn[i]), int(want_txn[i])) for i in bad[:20]]
    bad = np.nonzero(got_sig != want_sig)[0]
    assert len(bad) == 0, [(int(i), int(got_sig[i]), int(want_sig[i])) for i in bad[:20]]


def test_configs1_full_size():
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(1 << 20, synth.LARGE_NOOP, seed=1234)
    txn, sig = _run(payload, desc, nsig, 0)
    w_txn, w_sig = _expectation("avx512")(payload, desc, nsig)
    _check(txn, sig, w_txn, w_sig)
    assert (txn == 0).all() and np.array_equal(txn, expect)


@pytest.mark.parametrize("variant,sem", [("avx512", 0), ("portable", 1)])
def test_configs2_full_size(variant, sem):
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(1 << 20, synth.LARGE_NOOP, 1, 0.1, seed=4321)
    spliced = _splice_edges(payload, desc, 0.015, seed=5)
    txn, sig = _run(payload, desc, nsig, sem)
    w_txn, w_sig = _expectation(variant)(payload, desc, nsig)
    _check(txn, sig, w_txn, w_sig)
    codes = dict(zip(*np.unique(txn, return_counts=True)))
    # every failure class is present at full size
    assert all(codes.get(c, 0) > 1000 for c in (-1, -2, -3)) and codes[0] > 800_000, codes
    assert spliced > 15000


def test_configs3_full_size():
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(1 << 18, synth.MULTI, 12, 0.1, seed=777)
    txn, sig = _run(payload, desc, nsig, 0)
    w_txn, w_sig = _expectation("avx512")(payload, desc, nsig)
    _check(txn, sig, w_txn, w_sig)
    assert np.array_equal(txn, expect) and nsig > 1_500_000


def _run_device(payload, desc, nsig):
    """The HBM-resident form bench.py times: one launch over the whole batch (1M signatures: the
    carry-folded fd_dsm_kernel<1>; 64K: the one-lane latency path), per-signature codes too."""
    import torch
    import firedancer_amd as fa
    n = len(desc)
    eng = fa.Engine(device=0, max_txn=n, max_sig=nsig)
    try:
        pd = torch.from_numpy(payload).cuda()
        dd = torch.from_numpy(desc.view(np.uint8)).cuda()
        to = torch.empty(n, dtype=torch.int8, device="cuda")
        so = torch.empty(nsig, dtype=torch.int8, device="cuda")
        eng.verify_txns_device(pd.data_ptr(), dd.data_ptr(), n, nsig, to.data_ptr(), so.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return to.cpu().numpy(), so.cpu().numpy()
    finally:
        eng.close()


def test_configs0_full_size():
    """BASELINE configs[0]: 65,536 x 200-byte messages in one batch (the one-lane latency path)."""
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(1 << 16, synth.SMALL_MSG, 1, 0.1, seed=99)
    txn, sig = _run_device(payload, desc, nsig)
    w_txn, w_sig = _expectation("avx512")(payload, desc, nsig)
    _check(txn, sig, w_txn, w_sig)
    assert np.array_equal(txn, expect)


def test_configs2_full_size_device():
    """configs[2] in the form the headline is measured in: one HBM-resident 1M launch."""
    from firedancer_amd import synth
    payload, desc, expect, nsig = synth.make_batch(1 << 20, synth.LARGE_NOOP, 1, 0.1, seed=2468)
    spliced = _splice_edges(payload, desc, 0.015, seed=7)
    txn, sig = _run_device(payload, desc, nsig)
    w_txn, w_sig = _expectation("avx512")(payload, desc, nsig)
    _check(txn, sig, w_txn, w_sig)
    assert spliced > 15000
