"""CPU: pin the oracle (C restatement) to the reference's own outputs (tests/golden)."""
import hashlib

import numpy as np
import pytest

from oracle.oracle import SEM_AVX512, SEM_REF
from tests.golden_io import txns_fixture, vectors_as_txns

L_ORDER = 2**252 + 27742317777372353535851937790883648493


@pytest.mark.parametrize("sem,key", [(SEM_AVX512, "code_avx"), (SEM_REF, "code_ref")])
def test_vectors_single(oracle, golden, sem, key):
    v = golden["vectors"]
    bad = []
    for i in range(len(v["msg_sz"])):
        m = v["msg_arena"][v["msg_off"][i]: v["msg_off"][i] + v["msg_sz"][i]].tobytes()
        rc = oracle.verify(m, v["sig"][i].tobytes(), v["pub"][i].tobytes(), sem)
        if rc != v[key][i]:
            bad.append((int(v["set_id"][i]), int(v["tc_id"][i]), rc, int(v[key][i])))
    assert not bad, bad[:10]


@pytest.mark.parametrize("sem,key", [(SEM_AVX512, "code_avx"), (SEM_REF, "code_ref")])
def test_vectors_via_batch_layout(oracle, golden, sem, key):
    v = golden["vectors"]
    payload, desc = vectors_as_txns(v)
    txn_out, sig_out = oracle.verify_txns(payload, desc, len(desc), sem=sem, threads=4)
    np.testing.assert_array_equal(txn_out, v[key])
    np.testing.assert_array_equal(sig_out, v[key])


@pytest.mark.parametrize("sem,sfx", [(SEM_AVX512, "avx"), (SEM_REF, "ref")])
def test_txns(oracle, golden, sem, sfx):
    t = golden["txns"]
    payload, desc, nsig = txns_fixture(t)
    txn_out, sig_out = oracle.verify_txns(payload, desc, nsig, sem=sem, threads=4)
    np.testing.assert_array_equal(txn_out, t[f"txn_code_{sfx}"])
    np.testing.assert_array_equal(sig_out, t[f"sig_code_{sfx}"])


def test_batch_single_msg_api(oracle, golden):
    """oracle_ed25519_verify_batch_single_msg (two-pass structure) == reference batch codes."""
    t = golden["txns"]
    payload, desc, _ = txns_fixture(t)
    for i, dd in enumerate(desc):
        d = {k: int(dd[k]) for k in desc.dtype.names}
        if d["payload_sz"] < d["message_off"] or d["sig_cnt"] == 0 or d["sig_cnt"] > 16:
            continue
        if d["signature_off"] + 64 * d["sig_cnt"] > d["payload_sz"]:
            continue
        base = d["payload_off"]
        msg = payload[base + d["message_off"]: base + d["payload_sz"]].tobytes()
        sigs = payload[base + d["signature_off"]: base + d["signature_off"] + 64 * d["sig_cnt"]].tobytes()
        pubs = payload[base + d["acct_addr_off"]: base + d["acct_addr_off"] + 32 * d["sig_cnt"]].tobytes()
        assert oracle.verify_batch_single_msg(msg, sigs, pubs, d["sig_cnt"]) == t["txn_code_avx"][i]
    assert oracle.verify_batch_single_msg(b"", b"", b"", 0) == -1
    assert oracle.verify_batch_single_msg(b"", bytes(64 * 17), bytes(32 * 17), 17) == -1


def test_sha_and_k(oracle, golden):
    s = golden["sha"]
    for i, (off, sz) in enumerate(s["off"]):
        data = s["arena"][off: off + sz].tobytes()
        h = oracle.sha512(data)
        assert h == s["digest"][i].tobytes() == hashlib.sha512(data).digest()
        assert oracle.scalar_reduce(h) == s["k"][i].tobytes()


def test_scalar_reduce_extremes(oracle):
    rng = np.random.default_rng(5)
    cases = [bytes(64), b"\xff" * 64, (L_ORDER).to_bytes(64, "little"), (L_ORDER - 1).to_bytes(64, "little"),
             (L_ORDER * (2**259 // L_ORDER)).to_bytes(64, "little")]
    cases += [rng.integers(0, 256, 64, dtype=np.uint8).tobytes() for _ in range(500)]
    for c in cases:
        assert int.from_bytes(oracle.scalar_reduce(c), "little") == int.from_bytes(c, "little") % L_ORDER


def test_rfc8032_vector(oracle):
    prv = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    pub = oracle.public_from_private(prv)
    assert pub.hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    sig = oracle.sign(b"", pub, prv)
    assert sig.hex() == ("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e06522490155"
                         "5fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert oracle.verify(b"", sig, pub) == 0
