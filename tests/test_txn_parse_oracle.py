"""The fd_txn_parse restatement (oracle/fd_txn_oracle.c) against the
reference parser's recorded outputs (tests/golden/txn_parse.npz, made by
tests/golden/gen_txn_parse.py from src/ballet/txn/fd_txn_parse.c)."""
import os
import sys
import zlib

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import txn_builder as tb  # noqa: E402

STRIDE = 864


@pytest.fixture(scope="module")
def tg():
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "txn_parse.npz")))


def fixtures_from(tg):
    a, o, s = tg["fix_arena"], tg["fix_off"], tg["fix_sz"]
    return [a[o[i]: o[i] + s[i]].tobytes() for i in range(len(o))]


def crcs(fp, img):
    return np.array([zlib.crc32(img[i, : fp[i]].tobytes()) for i in range(len(fp))], np.uint32)


def test_reference_fixtures(oracle, tg):
    # test_txn_parse.c:259-265: footprints 852 / sizeof(fd_txn_t) / 0 / footprint(1,0)
    fx = fixtures_from(tg)
    fp, img = oracle.txn_parse_batch(*tb.pack(fx), STRIDE)
    assert fp.tolist() == tg["fix_fp"].tolist() == [90, 64, 852, 20, 0, 30]
    for i in range(len(fx)):
        assert img[i, : fp[i]].tobytes() == tg["fix_img"][i, : fp[i]].tobytes()


def test_txn1_fields(oracle, tg):
    # spot checks of test_txn_parse.c:txn1_correctness (:35-79)
    fp, img = oracle.txn_parse(fixtures_from(tg)[0])
    b = np.frombuffer(img, np.uint8)
    assert b[0] == 0xff and b[1] == 4                       # legacy, 4 signatures
    assert b[6] == 1 and b[7] == 11                         # ro signed / unsigned
    assert int(b[8]) | int(b[9]) << 8 == 23                 # acct_addr_cnt
    assert int(b[18]) | int(b[19]) << 8 == 7                # instr_cnt
    assert b[20] == 20 and b[20 + 6 * 10] == 22             # ix[0].program_id, ix[6].program_id


def test_mutation_sweep(oracle, tg):
    cases = tb.sweep_cases(fixtures_from(tg))
    fp, img = oracle.txn_parse_batch(*tb.pack(cases), STRIDE)
    assert np.array_equal(fp, tg["sweep_fp"])
    assert np.array_equal(crcs(fp, img), tg["sweep_crc"])


def test_builder_cases(oracle, tg):
    cases = tb.builder_cases()
    fp, img = oracle.txn_parse_batch(*tb.pack(cases), STRIDE)
    assert np.array_equal(fp, tg["build_fp"])
    assert np.array_equal(crcs(fp, img), tg["build_crc"])
