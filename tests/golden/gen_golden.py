#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE build (oracle/_ref).

Run in the build container only (needs /root/reference for
``make -C oracle ref``).  Every expected result code in the fixtures comes
from the reference's own fd_ed25519_verify / fd_ed25519_verify_batch_single_msg
compiled from its sources: ``code_avx`` from the AVX-512 (r43x6) build,
``code_ref`` from the portable build.  Inputs:

* ``cctv``, ``wycheproof``: the reference's known-answer tables
  (src/ballet/ed25519/test_ed25519_cctv.c, test_ed25519_wycheproof.c),
  exported by oracle/dump_vectors.c;
* ``malleability``: src/ballet/ed25519/test_ed25519_signature_malleability_
  should_{fail,pass}.bin (96-byte sig||pub records, message "Zcash");
* ``fuzz``: corpus/fuzz_ed25519_sigverify/* (prv[32]||msg, signed by the
  reference's fd_ed25519_sign, as fuzz_ed25519_sigverify.c does);
* ``edge``: small-order and non-canonical point encodings used as A and as
  R, plus S boundary values (SURVEY.md §8a edge table);
* ``random``: seeded valid signatures and mutations (bit flips, S+l,
  random/small-order R and A, message changes), messages 0..1232 bytes;
* ``txns``: multi-signer transactions (0..17 signers, wire layout of
  src/ballet/txn) with injected failures, expected per-transaction code
  from fd_ed25519_verify_batch_single_msg.
* ``sha``: SHA-512(R||A||M) and k = SHA-512 mod l for 256 inputs.

The fixtures are data only (inputs + expected outputs)."""
from __future__ import annotations

import hashlib
import os
import random
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.oracle import Reference, build  # noqa: E402

REFSRC = "/root/reference"
L_ORDER = 2**252 + 27742317777372353535851937790883648493
P = 2**255 - 19
B_ENC = bytes([0x58] + [0x66] * 31)
SET_IDS = {"cctv": 0, "wycheproof": 1, "malleability": 2, "fuzz": 3, "edge": 4, "random": 5}


def le(n: int) -> bytes:
    return n.to_bytes(32, "little")


def main() -> None:
    build(ref=True)
    ra, rp = Reference("avx512"), Reference("portable")
    vecs = []  # (set, tc_id, ok, msg, pub, sig)

    out = subprocess.run([os.path.join(ROOT, "oracle/_ref/dump_vectors")], check=True,
                         capture_output=True, text=True).stdout
    for line in out.splitlines():
        s, tc, ok, m, pub, sig = line.split()
        vecs.append((s, int(tc), int(ok), b"" if m == "-" else bytes.fromhex(m), bytes.fromhex(pub), bytes.fromhex(sig)))

    d = os.path.join(REFSRC, "src/ballet/ed25519")
    for name, ok in (("test_ed25519_signature_malleability_should_fail.bin", 0),
                     ("test_ed25519_signature_malleability_should_pass.bin", 1)):
        raw = open(os.path.join(d, name), "rb").read()
        for i in range(len(raw) // 96):
            rec = raw[96 * i: 96 * i + 96]
            vecs.append(("malleability", i + (0 if ok == 0 else 1000), ok, b"Zcash", rec[64:], rec[:64]))

    cdir = os.path.join(REFSRC, "corpus/fuzz_ed25519_sigverify")
    for i, fn in enumerate(sorted(os.listdir(cdir))):
        raw = open(os.path.join(cdir, fn), "rb").read()
        if len(raw) < 32:
            continue
        prv, msg = raw[:32], raw[32:]
        pub = ra.public_from_private(prv)
        vecs.append(("fuzz", i, 1, msg, pub, ra.sign(msg, pub, prv)))

    # edge encodings: small-order y values with both sign bits, y = p+k (non-canonical)
    y0 = int.from_bytes(bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"), "little")
    encs = []
    for y in (1, P - 1, 0, y0, P - y0):
        for sgn in (0, 1):
            encs.append(le(y | (sgn << 255)))
    for k in range(19):
        for sgn in (0, 1):
            encs.append(le((P + k) | (sgn << 255)))
    msg = b"edge"
    tc = 0
    for e in encs:
        vecs.append(("edge", tc, -1, msg, e, B_ENC + le(1))); tc += 1       # as A
        vecs.append(("edge", tc, -1, msg, B_ENC, e + le(1))); tc += 1       # as R
    for s in (0, 1, L_ORDER - 1, L_ORDER, L_ORDER + 1, 2**253 - 1, 2**253, 2**256 - 1, L_ORDER + 2**252):
        vecs.append(("edge", tc, -1, msg, B_ENC, B_ENC + le(s % 2**256))); tc += 1

    rng = random.Random(1234)
    small = [le(1), le(0), le(y0), le(P - 1), le(P - y0) , le(1 | 1 << 255)]
    for i in range(2000):
        prv = bytes(rng.getrandbits(8) for _ in range(32))
        msz = rng.choice([0, 1, 31, 32, 63, 64, 111, 112, 127, 128, 200, 1167]) if rng.random() < 0.3 else rng.randint(0, 400)
        msg = bytes(rng.getrandbits(8) for _ in range(msz))
        pub = ra.public_from_private(prv)
        sig = bytearray(ra.sign(msg, pub, prv))
        pub = bytearray(pub)
        kind = rng.randint(0, 12)
        if kind == 1:
            sig[rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif kind == 2:
            sig[32 + rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif kind == 3:
            pub[rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif kind == 4:
            msg = msg + b"\x01" if rng.random() < 0.5 or not msg else bytes([msg[0] ^ 0x80]) + msg[1:]
        elif kind == 5:
            sig[32:] = le((int.from_bytes(sig[32:], "little") + L_ORDER) % 2**256)
        elif kind == 6:
            sig[:32] = bytes(rng.getrandbits(8) for _ in range(32))
        elif kind == 7:
            pub[:] = bytes(rng.getrandbits(8) for _ in range(32))
        elif kind == 8:
            sig[32:] = bytes(rng.getrandbits(8) for _ in range(32))
        elif kind == 9:
            sig[:32] = rng.choice(small)
        elif kind == 10:
            pub[:] = rng.choice(small)
        elif kind == 11:
            sig[63] &= 0x0f  # S below 2^252: still canonical, wrong value
        vecs.append(("random", i, 1 if kind == 0 else -1, msg, bytes(pub), bytes(sig)))

    n = len(vecs)
    arena = bytearray()
    msg_off = np.zeros(n, np.uint32); msg_sz = np.zeros(n, np.uint32)
    pubs = np.zeros((n, 32), np.uint8); sigs = np.zeros((n, 64), np.uint8)
    code_avx = np.zeros(n, np.int8); code_ref = np.zeros(n, np.int8)
    set_id = np.zeros(n, np.uint8); tc_id = np.zeros(n, np.uint32); okf = np.zeros(n, np.int8)
    for i, (s, tc, ok, m, pub, sig) in enumerate(vecs):
        msg_off[i] = len(arena); msg_sz[i] = len(m); arena += m
        pubs[i] = np.frombuffer(pub, np.uint8); sigs[i] = np.frombuffer(sig, np.uint8)
        code_avx[i] = ra.verify(m, sig, pub); code_ref[i] = rp.verify(m, sig, pub)
        set_id[i] = SET_IDS[s]; tc_id[i] = tc; okf[i] = ok
        if ok in (0, 1):
            assert (code_avx[i] == 0) == (ok == 1), (s, tc)
            assert (code_ref[i] == 0) == (ok == 1), (s, tc)
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), msg_arena=np.frombuffer(bytes(arena), np.uint8),
                        msg_off=msg_off, msg_sz=msg_sz, pub=pubs, sig=sigs, code_avx=code_avx,
                        code_ref=code_ref, set_id=set_id, tc_id=tc_id, ok=okf)
    print("vectors:", n, {k: int((set_id == v).sum()) for k, v in SET_IDS.items()})

    # --- multi-signer transactions ---------------------------------------------------
    rng = random.Random(4321)
    payload = bytearray(); descs = []; sig_base = 0
    keys = []
    for _ in range(24):
        prv = bytes(rng.getrandbits(8) for _ in range(32))
        keys.append((prv, ra.public_from_private(prv)))
    for t in range(400):
        n_sig = rng.choice(list(range(0, 18)) + [1, 2, 4, 8, 12] * 4)
        signers = [keys[rng.randrange(len(keys))] for _ in range(n_sig)]
        body = bytearray([n_sig & 0xff, 0, 0, n_sig + 1])
        for _, pub in signers:
            body += pub
        body += bytes(rng.getrandbits(8) for _ in range(32 + 32))   # extra account + blockhash
        body += bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 1232 - 1 - 64 * n_sig - len(body)) if 1232 - 1 - 64 * n_sig - len(body) > 0 else 0))
        sigs_b = bytearray()
        for prv, pub in signers:
            sigs_b += ra.sign(bytes(body), pub, prv)
        # inject failures
        if n_sig and rng.random() < 0.5:
            j = rng.randrange(n_sig); kind = rng.randint(0, 5)
            if kind == 0:
                sigs_b[64 * j + rng.randrange(32)] ^= 1
            elif kind == 1:
                sigs_b[64 * j + 32: 64 * j + 64] = le((int.from_bytes(sigs_b[64 * j + 32: 64 * j + 64], "little") + L_ORDER) % 2**256)
            elif kind == 2:
                body[4 + 32 * j: 4 + 32 * j + 32] = small[rng.randrange(len(small))]
            elif kind == 3:
                sigs_b[64 * j: 64 * j + 32] = small[rng.randrange(len(small))]
            elif kind == 4:
                body[-1] ^= 0x55
            else:
                body[4 + 32 * j] ^= 0x10
        txn = bytes([n_sig]) + bytes(sigs_b) + bytes(body)
        while len(payload) % 8 != (t % 8):   # vary alignment of payloads
            payload += b"\xa5"
        off = len(payload); payload += txn
        msg_off_t = 1 + 64 * n_sig
        descs.append((off, sig_base, len(txn), msg_off_t, msg_off_t + 4, 1, n_sig))
        sig_base += n_sig
    # a few malformed descriptors (bounds) -> ERR_SIG
    for (off, sb, sz, mo, ao, so, ns) in list(descs[:4]):
        descs.append((off, sig_base, 10 if ns else 0, mo, ao, so, ns)); sig_base += ns
    dt = np.dtype([("payload_off", "<u4"), ("sig_base", "<u4"), ("payload_sz", "<u2"), ("message_off", "<u2"),
                   ("acct_addr_off", "<u2"), ("signature_off", "u1"), ("sig_cnt", "u1")])
    desc = np.array(descs, dtype=dt)
    assert desc.itemsize == 16
    pay = np.frombuffer(bytes(payload) + bytes(256), np.uint8).copy()
    t_avx, s_avx = ra.verify_txns(pay, desc, sig_base)
    t_ref, s_ref = rp.verify_txns(pay, desc, sig_base)
    np.savez_compressed(os.path.join(HERE, "txns.npz"), payload=pay, desc=desc.view(np.uint8).reshape(-1, 16),
                        sig_total=np.array([sig_base]), txn_code_avx=t_avx, txn_code_ref=t_ref,
                        sig_code_avx=s_avx, sig_code_ref=s_ref)
    print("txns:", len(desc), "sigs:", sig_base, "txn codes:", np.unique(t_avx, return_counts=True))

    # --- SHA-512 / k vectors ----------------------------------------------------------
    rng = random.Random(99)
    ins, outs, ks = [], [], []
    arena = bytearray(); offs = []
    for i in range(256):
        m = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 1300)))
        data = bytes(rng.getrandbits(8) for _ in range(64)) + m
        h = ra.sha512(data)
        assert h == hashlib.sha512(data).digest()
        offs.append((len(arena), len(data))); arena += data
        outs.append(np.frombuffer(h, np.uint8))
        ks.append(np.frombuffer(le(int.from_bytes(h, "little") % L_ORDER), np.uint8))
    np.savez_compressed(os.path.join(HERE, "sha.npz"), arena=np.frombuffer(bytes(arena), np.uint8),
                        off=np.array(offs, np.uint32), digest=np.array(outs), k=np.array(ks))
    print("sha vectors: 256")


if __name__ == "__main__":
    main()
