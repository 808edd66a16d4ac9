"""Signatures whose public key A and / or commitment R carry a torsion component (test vectors).

The half-size check (firedancer_amd/csrc/fd_gpu_lattice.h) is equivalent to the reference's cofactorless
R == [S]B - [k]A only because the lattice modulus is 8l and c1 is odd; both matter exactly when A or R has
a component in the 8-torsion subgroup.  The reference (fd_ed25519_user.c:204-226) accepts such a signature
only if the torsion parts cancel exactly:

  A = [a]B + T,  R = [r]B + T',  S = r + k a mod l   ->   [S]B - [k]A - R = -[k]T - T'

so it returns SUCCESS iff T' == -[k]T, else ERR_MSG (A and R are not small order, they decode, S < l).
make_cases() builds all four kinds -- A mixed / R clean, A clean / R mixed, both mixed and cancelling,
both mixed and not -- with plain Python integer arithmetic on edwards25519 (RFC 8032 formulas), SHA-512
from hashlib.  Test data only; the expected codes are re-derived by the oracle / the compiled reference
in the tests.
"""
import hashlib
import random

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)

IDENT = (0, 1, 1, 0)


def _add(p, q):                          # extended coordinates, a = -1 (RFC 8032 5.1.4)
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = 2 * D * t1 * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _mul(k, p):
    q = IDENT
    while k:
        if k & 1:
            q = _add(q, p)
        p = _add(p, p)
        k >>= 1
    return q


def _neg(p):
    return ((-p[0]) % P, p[1], p[2], (-p[3]) % P)


def _affine(p):
    zi = pow(p[2], P - 2, P)
    return p[0] * zi % P, p[1] * zi % P


def _eq(p, q):
    return (p[0] * q[2] - q[0] * p[2]) % P == 0 and (p[1] * q[2] - q[1] * p[2]) % P == 0


def _recover_x(y, sign):
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    if (v * x * x - u) % P:
        if (v * x * x + u) % P:
            return None
        x = x * SQRTM1 % P
    if (x & 1) != sign:
        x = (-x) % P
    return x


def encode(p):
    x, y = _affine(p)
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def _point(y, sign):
    x = _recover_x(y, sign)
    return None if x is None else (x, y, 1, x * y % P)


BASE = _point(4 * pow(5, P - 2, P) % P, 0)


def torsion8(rng):
    """The 8 points of the torsion subgroup, T8[i] = [i]T for a point T of order 8."""
    while True:
        p = _point(rng.randrange(P), rng.randrange(2))
        if p is None:
            continue
        t = _mul(L, p)                   # the torsion component of a random point
        if not _eq(_mul(4, t), IDENT):   # order exactly 8
            out, q = [], IDENT
            for _ in range(8):
                out.append(q)
                q = _add(q, t)
            return out


def _k(r_enc, a_enc, msg):
    return int.from_bytes(hashlib.sha512(r_enc + a_enc + msg).digest(), "little") % L


def make_cases(n_per_kind=64, seed=20261017):
    """-> list of (msg, sig64, pub32, expected_code, kind)."""
    rng = random.Random(seed)
    t8 = torsion8(rng)
    out = []
    for kind in ("A_mixed", "R_mixed", "both_cancel", "both_mixed"):
        made = 0
        while made < n_per_kind:
            a, r = rng.randrange(1, L), rng.randrange(1, L)
            ti = rng.randrange(1, 8) if kind != "R_mixed" else 0
            A = _add(_mul(a, BASE), t8[ti])
            a_enc = encode(A)
            msg = rng.randbytes(rng.randrange(0, 200))
            if kind == "both_cancel":
                # find R's torsion T' == -[k]T: k depends on R's encoding, so try each T' (1 in 8 matches)
                rb = _mul(r, BASE)
                hit = None
                for tj in range(8):
                    r_enc = encode(_add(rb, t8[tj]))
                    k = _k(r_enc, a_enc, msg)
                    if _eq(_add(t8[tj], _mul(k, t8[ti])), IDENT):
                        hit = (r_enc, k)
                        break
                if hit is None or hit[0] == encode(rb):
                    continue                 # only the T' = O solution: not a torsion case
                r_enc, k = hit
            else:
                tj = rng.randrange(1, 8) if kind in ("R_mixed", "both_mixed") else 0
                r_enc = encode(_add(_mul(r, BASE), t8[tj]))
                k = _k(r_enc, a_enc, msg)
            s = (r + k * a) % L
            lhs = _add(_mul(s, BASE), _neg(_mul(k, A)))          # [S]B - [k]A
            code = 0 if _eq(lhs, _point_from_enc(r_enc)) else -3
            out.append((msg, r_enc + s.to_bytes(32, "little"), a_enc, code, kind))
            made += 1
    return out


def _point_from_enc(enc):
    v = int.from_bytes(enc, "little")
    return _point(v & ((1 << 255) - 1), v >> 255)
