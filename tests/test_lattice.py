"""Half-size scalars (firedancer_amd/csrc/fd_gpu_lattice.h), the device reduction compiled as host C.

The verification rewrite Q = [c1 S mod l]B + [c0](-A) + [c1](-R) == O is equivalent to the reference's
R == [S]B - [k]A (fd_ed25519_user.c:204-226) exactly when c0 == c1 k (mod 8l) and c1 is odd with
0 < |c1| < l.  Every pair the reduction returns must satisfy that (checked here with Python integers);
pairs it cannot bound go to the full-length walk, and that must be rare for hash-distributed k.
The GPU tests cover the kernels end to end against the oracle and the compiled reference."""
import ctypes
import os
import random

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 2**252 + 27742317777372353535851937790883648493
N8L = 8 * L


@pytest.fixture(scope="module")
def lat():
    from firedancer_amd import build
    return ctypes.CDLL(build.build_lattice_host())


def _run(lib, k):
    kw = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xffffffff for i in range(8)])
    c0 = (ctypes.c_uint32 * 5)()
    c1 = (ctypes.c_uint32 * 5)()
    neg = ctypes.c_int()
    ok = lib.fd_lat_halfsize_host(c0, c1, ctypes.byref(neg), kw)
    v0 = sum(c0[i] << (32 * i) for i in range(5))
    v1 = sum(c1[i] << (32 * i) for i in range(5))
    return ok, v0, -v1 if neg.value else v1


def _check(k, c0, c1):
    assert (c0 - c1 * k) % N8L == 0, hex(k)
    assert c1 % 2 == 1 and 0 <= c0 < 2**159 and 0 < abs(c1) < 2**159, hex(k)


def test_random_k(lat):
    rng = random.Random(20261017)
    n, fails = 20000, 0
    for _ in range(n):
        k = rng.randrange(L)
        ok, c0, c1 = _run(lat, k)
        if ok:
            _check(k, c0, c1)
        else:
            fails += 1
    assert fails == 0, fails                   # within 2^159: none for hash-distributed k


@pytest.mark.parametrize("k", [0, 1, 2, 3, 12345, 2**64 - 1, 2**127, 2**128 - 1, 2**128, 2**128 + 1, 2**200,
                               2**252, L - 1, L - 2, (L - 1) // 2, N8L // 16])
def test_edge_k(lat, k):
    ok, c0, c1 = _run(lat, k)
    if ok:
        _check(k, c0, c1)
    if k < 2**128:
        assert ok and c0 == k and c1 == 1      # already short: (k, 1)


def test_no_short_odd_vector(lat):
    """k = l - 1: every lattice vector with odd c1 has c0 ~ l (c0 == l (c1 mod 8) - c1 mod 8l), so the
    reduction must refuse rather than return a long or even pair."""
    ok, _, _ = _run(lat, L - 1)
    assert not ok
