"""Torsion-component signatures (tests/torsion.py): the generator's expected codes are the reference's.

Checked here against the oracle restatement of the reference's verify (and the compiled reference when this
CPU runs its AVX-512 build), so the GPU test (test_gpu_torsion.py) can use them as the expectation."""
import collections

import pytest

from tests import torsion


@pytest.fixture(scope="module")
def cases():
    return torsion.make_cases(32)


def test_cases_match_oracle(cases, oracle):
    for msg, sig, pub, code, kind in cases:
        assert oracle.verify(msg, sig, pub) == code, kind


def test_cases_match_reference(cases):
    from oracle.oracle import Reference, cpu_has_avx512_ifma
    variants = ["portable"] + (["avx512"] if cpu_has_avx512_ifma() else [])
    try:
        refs = [Reference(v) for v in variants]
    except (FileNotFoundError, OSError):
        pytest.skip("oracle/_ref not built")
    for msg, sig, pub, code, kind in cases:
        for ref in refs:
            assert ref.verify(msg, sig, pub) == code, kind


def test_case_mix(cases):
    """Every kind is present; cancelling pairs verify, R-only torsion never does, and some A-only
    torsion signatures verify ([k]T = O) while most do not."""
    by = collections.defaultdict(collections.Counter)
    for *_, code, kind in cases:
        by[kind][code] += 1
    assert by["both_cancel"] == {0: 32}
    assert by["R_mixed"] == {-3: 32}
    assert by["A_mixed"][-3] > 16 and by["both_mixed"][-3] > 16
