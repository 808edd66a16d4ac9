"""CPU: the canonical packing procedure of fd_gpu_f25519.h fe_pack (one carry pass, then subtract p iff
h + 19 >= 2^255), restated limb for limb in Python, equals the value mod p for every input the device can
give it (limbs below 2^31).  This pins the claim that a second carry pass is unnecessary
(profiles/r03/pack_onepass)."""
import random

W = [26, 25] * 5
S = [sum(W[:i]) for i in range(10)]
P = 2**255 - 19
M32 = (1 << 32) - 1


def _val(h):
    return sum(h[i] << S[i] for i in range(10))


def fe_pack_model(a):
    h = list(a)
    for i in range(9):                                    # one carry pass, u32 arithmetic
        h[i + 1] = (h[i + 1] + (h[i] >> W[i])) & M32
        h[i] &= (1 << W[i]) - 1
    h[0] = (h[0] + 19 * (h[9] >> 25)) & M32
    h[9] &= (1 << 25) - 1
    q = (h[0] + 19) >> 26
    for i in range(1, 10):
        q = (h[i] + q) >> W[i]
    h[0] = (h[0] + 19 * q) & M32
    for i in range(9):
        h[i + 1] = (h[i + 1] + (h[i] >> W[i])) & M32
        h[i] &= (1 << W[i]) - 1
    h[9] &= (1 << 25) - 1
    return _val(h)


def _limbs(x):
    a = [(x >> S[i]) & ((1 << W[i]) - 1) for i in range(10)]
    a[9] = min(x >> S[9], (1 << 31) - 1)
    return a


def test_fe_pack_one_pass_is_canonical():
    rng = random.Random(1)
    cases = [[(1 << 31) - 1] * 10, [0] * 10]
    cases += [_limbs(x) for x in (P - 1, P, P + 1, 2 * P - 1, 2 * P, 2**255 - 1, 2**255, 2**255 + 18, 19)]
    for _ in range(20000):
        m = rng.randrange(3)
        if m == 0:
            cases.append([rng.randrange(1 << 31) for _ in range(10)])
        elif m == 1:
            cases.append([(1 << 31) - 1 - rng.randrange(4) for _ in range(10)])
        else:
            cases.append([((1 << W[i]) - 1) + rng.randrange(1 << rng.randrange(1, 6)) for i in range(10)])
    for a in cases:
        assert fe_pack_model(a) == _val(a) % P, a
