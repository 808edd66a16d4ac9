#!/usr/bin/env python3
"""Generate tests/golden/hs_top.npz: valid 1232-byte single-signer transactions whose
half-size scalars (c0, c1) (firedancer_amd/csrc/fd_gpu_lattice.h) both lie below 2^120,
so their top nonzero radix-16 window is < 30.

Why these inputs matter: the half-size walk Q = [s']B + [c0](-A) + [c1](-R) adds the
radix-2^16 digits of s' at windows 0..30 (digit j at window 4j, digit j+8 at window
4j+2).  A walk that starts at the top window of c0 / c1 alone skips the base-point
digits above it, so a wave whose every pending signature has such small scalars --
one signature alone in a batch, or in the last wave of a batch -- rejected a valid
signature with ERR_MSG.  For hash-distributed k that happens for ~7.5e-6 of signatures
(host histogram over 400K random k: top 29 in 3, 30 in 528, 31 in 136,517, 32 in
262,217), which is why only a long stream run ever met one (round 4's withheld frags).

Each transaction is a synthetic LARGE_NOOP txn (fd_benchg.c large_noop_t layout, from
firedancer_amd/synth.py) with its last 8 payload bytes (instruction data) replaced by a
counter, re-signed with the oracle's signer (the fd_ed25519_sign restatement), kept when
the lattice reduction (compiled for the host, as tests/test_lattice.py does) gives
top < 30.  The expected code of every one is the reference's: FD_ED25519_SUCCESS from
the AVX-512 and the portable builds of fd_ed25519_verify (oracle/_ref), checked here.

Run in the build container: python tests/golden/gen_hs_top.py  (about a minute on 8 CPUs).
The fixture is data only (inputs + expected outputs)."""
from __future__ import annotations

import ctypes
import hashlib
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

L = 2**252 + 27742317777372353535851937790883648493
WANT = 8                 # transactions to find
TOP_MAX = 29             # top window of (c0, c1) at most this


def _digits(v: int, n: int = 40) -> list[int]:
    out, c = [], 0
    for i in range(n):
        x = ((v >> (4 * i)) & 15) + c
        c = (x + 8) >> 4 if i < n - 1 else 0
        out.append(x - (c << 4))
    return out


def _top(lib, k: int):
    kw = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xffffffff for i in range(8)])
    c0 = (ctypes.c_uint32 * 5)(); c1 = (ctypes.c_uint32 * 5)(); neg = ctypes.c_int()
    if not lib.fd_lat_halfsize_host(c0, c1, ctypes.byref(neg), kw):
        return None
    v0 = sum(c0[i] << (32 * i) for i in range(5)); v1 = sum(c1[i] << (32 * i) for i in range(5))
    da, dr = _digits(v0), _digits(v1)
    return max([j for j in range(40) if da[j] or dr[j]] + [0])


def _search(args):
    start, count = args
    from firedancer_amd import build, synth
    from oracle.oracle import Oracle
    lib = ctypes.CDLL(build.build_lattice_host())
    o = Oracle()
    keys = synth.keys(1, 20261018)
    prv, pub = keys[0, 0:32].tobytes(), keys[0, 32:64].tobytes()
    payload, desc, _, _ = synth.make_batch(1, synth.LARGE_NOOP, seed=20261018, key_arr=keys, threads=1)
    d = desc[0]
    base = bytearray(payload[:int(d["payload_sz"])].tobytes())
    so, mo = int(d["signature_off"]), int(d["message_off"])
    hits = []
    for ctr in range(start, start + count):
        base[-8:] = ctr.to_bytes(8, "little")
        msg = bytes(base[mo:])
        sig = o.sign(msg, pub, prv)
        k = int.from_bytes(hashlib.sha512(sig[:32] + pub + msg).digest(), "little") % L
        t = _top(lib, k)
        if t is not None and t <= TOP_MAX:
            txn = bytearray(base); txn[so:so + 64] = sig
            hits.append((ctr, t, bytes(txn)))
    return hits


def main() -> None:
    from firedancer_amd import synth
    from oracle.oracle import Reference
    step, hits, nxt = 40000, [], 0
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        while len(hits) < WANT:
            batch = [(nxt + i * step, step) for i in range(8)]
            nxt += 8 * step
            for h in pool.map(_search, batch):
                hits += h
            print(f"searched {nxt}: {len(hits)} found", flush=True)
    hits = sorted(hits)[:WANT]
    keys = synth.keys(1, 20261018)
    pub = keys[0, 32:64].tobytes()
    _, desc, _, _ = synth.make_batch(1, synth.LARGE_NOOP, seed=20261018, key_arr=keys, threads=1)
    d = desc[0]
    so, ao, mo = int(d["signature_off"]), int(d["acct_addr_off"]), int(d["message_off"])
    refs = {v: Reference(v) for v in ("avx512", "portable")}
    txns = np.zeros((len(hits), 1232), np.uint8)
    code = {v: np.zeros(len(hits), np.int8) for v in refs}
    for i, (_, _, t) in enumerate(hits):
        txns[i, :len(t)] = np.frombuffer(t, np.uint8)
        for v, r in refs.items():
            code[v][i] = r.verify(t[mo:], t[so:so + 64], t[ao:ao + 32])
        assert t[ao:ao + 32] == pub
    assert all((c == 0).all() for c in code.values()), code
    np.savez_compressed(os.path.join(HERE, "hs_top.npz"), txn=txns,
                        payload_sz=np.full(len(hits), 1232, np.uint16),
                        signature_off=np.full(len(hits), so, np.uint16), acct_addr_off=np.full(len(hits), ao, np.uint16),
                        message_off=np.full(len(hits), mo, np.uint16),
                        top=np.array([h[1] for h in hits], np.int8), counter=np.array([h[0] for h in hits], np.uint64),
                        code_avx=code["avx512"], code_ref=code["portable"])
    print("wrote hs_top.npz:", [(h[0], h[1]) for h in hits])


if __name__ == "__main__":
    main()
