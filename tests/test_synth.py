"""CPU: the synthetic transaction generator (host C) produces what the
reference verifier (via the oracle) expects."""
import numpy as np
import pytest

from firedancer_amd import synth


@pytest.mark.parametrize("kind,ms,inv", [(synth.LARGE_NOOP, 1, 0.0), (synth.SMALL_MSG, 1, 0.0),
                                         (synth.LARGE_NOOP, 1, 0.5), (synth.MULTI, 12, 0.3)])
def test_synth_matches_oracle(oracle, kind, ms, inv):
    pay, desc, exp, ns = synth.make_batch(300, kind, ms, inv, seed=11)
    to, so = oracle.verify_txns(pay, desc, ns, threads=4)
    np.testing.assert_array_equal(to, exp)
    assert desc["sig_base"][-1] + desc["sig_cnt"][-1] == ns
    if kind == synth.LARGE_NOOP:
        assert (desc["payload_sz"] == 1232).all() and (desc["message_off"] == 65).all()
        assert (desc["acct_addr_off"] == 69).all()


def test_synth_deterministic():
    a = synth.make_batch(64, synth.LARGE_NOOP, seed=5)
    b = synth.make_batch(64, synth.LARGE_NOOP, seed=5)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
