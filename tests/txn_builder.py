"""Deterministic Solana wire-format transaction builder and mutators for the
fd_txn_parse parity tests (test data generation only).

Wire format (src/ballet/txn/fd_txn.h:1-130, fd_txn_parse.c:79-247):
  compact sig_cnt | sig_cnt x 64-B signature | [0x80|ver] (v0 only) |
  header (sig_cnt, ro_signed, ro_unsigned) | compact acct_cnt | acct_cnt x 32 B |
  32-B blockhash | compact instr_cnt | instr* | (v0) compact lut_cnt | lut*
  instr = program_id u8 | compact n | n x u8 account index | compact d | d bytes
  lut   = 32-B table key | compact nw | nw x u8 | compact nr | nr x u8

Every case set is a pure function of its seed, so the expected outputs in
tests/golden/txn_parse.npz (recorded from the reference parser) line up
with inputs regenerated here on any machine.
"""
from __future__ import annotations

import glob
import os

import numpy as np

MTU = 1232
FIXTURE_NAMES = [f"transaction{i}.bin" for i in range(1, 7)]
SWEEP_BASES = (0, 1, 2, 5)      # transaction1, 2, 3, 6
SWEEP_VALUES = (0x00, 0x01, 0x02, 0x7f, 0x80, 0x81, 0xfe, 0xff)
SWEEP_DELTAS = (1, -1, 2, -2, 0x80)


def cu16(v: int) -> bytes:
    """compact-u16 encoding (fd_compact_u16.h:89-103)."""
    out = bytearray([v & 0x7f])
    if v > 0x7f:
        out[0] |= 0x80
        out.append((v >> 7) & 0x7f)
        if v > 0x3fff:
            out[1] |= 0x80
            out.append(v >> 14)
    return bytes(out)


def build_txn(rng: np.random.Generator, v0: bool | None = None, max_sz: int = MTU) -> bytes:
    """One random, usually valid, transaction."""
    if v0 is None:
        v0 = bool(rng.integers(2))
    for _ in range(16):
        sig_cnt = int(rng.choice([1, 1, 1, 2, 2, 3, 4, 8, 12, 16]))
        ro_signed = int(rng.integers(sig_cnt))
        acct_cnt = int(rng.integers(sig_cnt + (1 if sig_cnt < 2 else 0), min(sig_cnt + 24, 128) + 1))
        acct_cnt = max(acct_cnt, 2)
        ro_unsigned = int(rng.integers(acct_cnt - sig_cnt + 1))
        luts = []
        if v0:
            for _ in range(int(rng.choice([0, 0, 1, 2, 3, 6]))):
                room = 128 - acct_cnt
                nw = int(rng.integers(0, min(room, 8) + 1))
                nr = int(rng.integers(0 if nw else 1, min(room, 8) + 1))
                luts.append((rng.bytes(32), rng.integers(0, 256, nw, dtype=np.uint8).tobytes(),
                             rng.integers(0, 256, nr, dtype=np.uint8).tobytes()))
            while acct_cnt + sum(len(w) + len(r) for _, w, r in luts) > 128:
                luts.pop()
        total_accts = acct_cnt + sum(len(w) + len(r) for _, w, r in luts)
        instrs = []
        for _ in range(int(rng.choice([0, 1, 1, 2, 3, 5, 8]))):
            prog = int(rng.integers(1, acct_cnt))
            n = int(rng.choice([0, 1, 2, 3, 6, 12]))
            accts = rng.integers(0, total_accts, n, dtype=np.uint8).tobytes()
            d = int(rng.choice([0, 1, 4, 9, 40, 130, 200]))
            instrs.append((prog, accts, rng.bytes(d)))
        msg = bytearray()
        if v0:
            msg.append(0x80)
        msg += bytes([sig_cnt, ro_signed, ro_unsigned])
        msg += cu16(acct_cnt) + rng.bytes(32 * acct_cnt) + rng.bytes(32)
        msg += cu16(len(instrs))
        for prog, accts, data in instrs:
            msg += bytes([prog]) + cu16(len(accts)) + accts + cu16(len(data)) + data
        if v0:
            msg += cu16(len(luts))
            for key, w, r in luts:
                msg += key + cu16(len(w)) + w + cu16(len(r)) + r
        txn = cu16(sig_cnt) + rng.bytes(64 * sig_cnt) + bytes(msg)
        if len(txn) <= max_sz:
            return txn
    return txn[:max_sz]


def mutate(rng: np.random.Generator, txn: bytes) -> bytes:
    b = bytearray(txn)
    kind = int(rng.integers(5))
    if kind == 0 and len(b) > 1:            # truncate
        return bytes(b[: int(rng.integers(len(b)))])
    if kind == 1:                           # append junk
        return bytes(b + rng.bytes(int(rng.integers(1, 4))))[:MTU + 2]
    for _ in range(int(rng.integers(1, 4))):  # byte rewrites, biased to the header
        if not b:
            break
        pos = int(rng.integers(min(len(b), 96))) if rng.integers(2) else int(rng.integers(len(b)))
        b[pos] = int(rng.choice([0, 1, 0x7f, 0x80, 0xff, int(rng.integers(256))]))
    return bytes(b)


def builder_cases(seed: int = 7, n: int = 6000) -> list[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        t = build_txn(rng)
        out.append(t if i % 3 == 0 else mutate(rng, t))
    return out


def sweep_cases(fixtures: list[bytes]) -> list[bytes]:
    """test_txn_parse.c:test_mutate-style single-byte rewrites + every truncation."""
    out = []
    for bi in SWEEP_BASES:
        base = fixtures[bi]
        for pos in range(len(base)):
            vals = set(SWEEP_VALUES) | {(base[pos] + d) & 0xff for d in SWEEP_DELTAS}
            vals.discard(base[pos])
            for v in sorted(vals):
                b = bytearray(base)
                b[pos] = v
                out.append(bytes(b))
    for base in fixtures:
        for ln in range(len(base)):
            out.append(base[:ln])
    return out


def load_reference_fixtures(ref_dir: str = "/root/reference/src/ballet/txn/fixtures") -> list[bytes]:
    return [open(os.path.join(ref_dir, f), "rb").read() for f in FIXTURE_NAMES]


def pack(cases: list[bytes], align: int = 16):
    """Arena + offsets + sizes (each payload 16-B aligned, 64 B of zero tail slack)."""
    off = np.zeros(len(cases), np.uint32)
    sz = np.zeros(len(cases), np.uint16)
    pos = 0
    for i, c in enumerate(cases):
        off[i] = pos
        sz[i] = len(c)
        pos += (len(c) + align - 1) // align * align
    arena = np.zeros(pos + 64, np.uint8)
    for i, c in enumerate(cases):
        arena[off[i]: off[i] + len(c)] = np.frombuffer(c, np.uint8)
    return arena, off, sz
