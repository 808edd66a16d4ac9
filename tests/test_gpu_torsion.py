"""GPU: signatures with a torsion component in A and / or R (tests/torsion.py), on every engine path.

This is where the half-size check (fd_gpu_lattice.h) could differ from the reference: with a lattice modulus
of l instead of 8l, or an even c1, torsion parts would be dropped and cofactor-only-valid signatures
accepted.  Expected codes: the reference's (pinned by tests/test_torsion.py)."""
import numpy as np
import pytest

from tests import torsion

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cases():
    return torsion.make_cases(64)


@pytest.mark.parametrize("sem", [0, 1])            # AVX-512 and portable semantics: the same codes here
def test_torsion_signatures(cases, engine_path, sem):
    import firedancer_amd as fa
    msgs = [c[0] for c in cases]
    sigs = [c[1] for c in cases]
    pubs = [c[2] for c in cases]
    want = np.array([c[3] for c in cases], np.int8)
    eng = fa.Engine(device=0, max_txn=len(cases), max_sig=len(cases), max_payload=1 << 20, semantics=sem)
    try:
        got = np.asarray(eng.verify_many(msgs, sigs, pubs), np.int8)
    finally:
        eng.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), cases[i][4], int(got[i]), int(want[i])) for i in bad[:10]]


def test_torsion_dropin(cases):
    """The link-level drop-in on the same inputs (one signature per call)."""
    import firedancer_amd as fa
    for msg, sig, pub, code, kind in cases[::8]:
        assert fa.fd_ed25519_verify(msg, sig, pub) == code, kind
