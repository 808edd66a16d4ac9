"""SHA-512 against the NIST CAVP vectors the reference tests with
(tests/golden/sha_cavp.npz from src/ballet/sha512/cavp): the oracle on CPU;
the GPU batch SHA-512 (fdgpu_sha512_batch_host, the fd_sha512_batch_*
replacement) on the GPU, plus random lengths / alignments vs hashlib."""
import hashlib
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def cavp():
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "sha_cavp.npz"))
    off = np.concatenate([[0], np.cumsum(d["lens"].astype(np.int64))[:-1]])
    msgs = [d["data"][o: o + n].tobytes() for o, n in zip(off, d["lens"])]
    return msgs, [d["md"][i].tobytes() for i in range(len(msgs))]


def test_oracle_sha512_cavp(oracle, cavp):
    msgs, mds = cavp
    assert len(msgs) == 257
    for m, md in zip(msgs, mds):
        assert oracle.sha512(m) == md == hashlib.sha512(m).digest()


@pytest.mark.gpu
def test_gpu_sha512_batch_cavp(cavp):
    from firedancer_amd.engine import sha512_batch
    msgs, mds = cavp
    assert sha512_batch(msgs) == mds


@pytest.mark.gpu
def test_gpu_sha512_batch_random():
    from firedancer_amd.engine import sha512_batch
    rng = np.random.default_rng(5)
    lens = list(range(0, 300)) + [int(x) for x in rng.integers(0, 5000, 700)] + [111, 112, 127, 128, 129, 239, 240]
    # unaligned starts: each message follows the previous one in one buffer
    msgs = [rng.bytes(n) for n in lens]
    assert sha512_batch(msgs) == [hashlib.sha512(m).digest() for m in msgs]
