"""GPU parity of the raw-payload path: the device fd_txn_parse
(fd_gpu_txn.h) against the reference parser's recorded outputs and the
oracle, and parse + verify of raw payloads against the oracle.  All
calls go through the C ABI (fdgpu_txn_parse_device,
fdgpu_ed25519_verify_raw_{host,device})."""
import os
import sys
import zlib

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import raw_expect  # noqa: E402
import txn_builder as tb  # noqa: E402

pytestmark = pytest.mark.gpu
STRIDE = 864


@pytest.fixture(scope="module")
def tg():
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "txn_parse.npz")))


def fixtures_from(tg):
    a, o, s = tg["fix_arena"], tg["fix_off"], tg["fix_sz"]
    return [a[o[i]: o[i] + s[i]].tobytes() for i in range(len(o))]


def gpu_parse(cases):
    import torch
    from firedancer_amd import engine
    arena, off, sz = tb.pack(cases)
    raw = np.zeros(len(cases), engine.RAW_DTYPE)
    raw["payload_off"] = off
    raw["payload_sz"] = sz
    d_arena = torch.from_numpy(arena).cuda()
    d_raw = torch.from_numpy(raw.view(np.uint8)).cuda()
    d_img = torch.full((len(cases), STRIDE), 0xAB, dtype=torch.uint8, device="cuda")
    d_fp = torch.zeros(len(cases), dtype=torch.int16, device="cuda")
    engine.txn_parse_device(d_arena.data_ptr(), d_raw.data_ptr(), len(cases), d_img.data_ptr(), d_fp.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_fp.cpu().numpy().view(np.uint16), d_img.cpu().numpy()


def crcs(fp, img):
    return np.array([zlib.crc32(img[i, : fp[i]].tobytes()) for i in range(len(fp))], np.uint32)


def test_parse_reference_fixtures(tg):
    fp, img = gpu_parse(fixtures_from(tg))
    assert fp.tolist() == tg["fix_fp"].tolist()
    for i in range(len(fp)):
        assert img[i, : fp[i]].tobytes() == tg["fix_img"][i, : fp[i]].tobytes()


def test_parse_mutation_sweep(tg):
    fp, img = gpu_parse(tb.sweep_cases(fixtures_from(tg)))
    np.testing.assert_array_equal(fp, tg["sweep_fp"])
    np.testing.assert_array_equal(crcs(fp, img), tg["sweep_crc"])


def test_parse_builder(tg):
    fp, img = gpu_parse(tb.builder_cases())
    np.testing.assert_array_equal(fp, tg["build_fp"])
    np.testing.assert_array_equal(crcs(fp, img), tg["build_crc"])


def test_parse_fuzz_vs_oracle(oracle):
    """Fresh seeded cases (not in the golden file), incl. oversize and empty payloads."""
    rng = np.random.default_rng(2024)
    cases = [b"", b"\x01", bytes(1233), bytes(rng.integers(0, 256, 1232, dtype=np.uint8))]
    for i in range(20000):
        t = tb.build_txn(rng)
        cases.append(tb.mutate(rng, t) if i % 2 else t)
    fp, img = gpu_parse(cases)
    ofp, oimg = oracle.txn_parse_batch(*tb.pack(cases), STRIDE)
    np.testing.assert_array_equal(fp, ofp)
    np.testing.assert_array_equal(crcs(fp, img), crcs(ofp, oimg))


def _raw_cases():
    """Valid signed txns (synth), adversarial mix, multi-signer, and parse failures."""
    from firedancer_amd import synth
    cases = []
    for kind, ms, inv, n, seed in ((synth.LARGE_NOOP, 1, 0.0, 600, 5), (synth.MULTI, 12, 0.3, 400, 6),
                                   (synth.SMALL_MSG, 1, 0.2, 400, 7)):
        payload, desc, _, _ = synth.make_batch(n, kind, ms, inv, seed=seed)
        for d in desc:
            cases.append(payload[d["payload_off"]: d["payload_off"] + d["payload_sz"]].tobytes())
    rng = np.random.default_rng(77)
    sigd = list(cases)
    for i in range(600):                       # mutate signed txns: parse failures and verify failures
        cases.append(tb.mutate(rng, sigd[int(rng.integers(len(sigd)))]))
    for i in range(600):                       # random structures (17+ signers, v0 tables, ...)
        cases.append(tb.build_txn(rng))
    return cases


@pytest.mark.parametrize("sem", [0, 1])
def test_verify_raw_host_vs_oracle(oracle, sem):
    from firedancer_amd import Engine
    cases = _raw_cases()
    arena, off, sz = tb.pack(cases)
    want, wfp, wimg = raw_expect.expected_codes(oracle, arena, off, sz, sem=sem)
    eng = Engine(device=0, max_txn=len(cases), max_sig=16 * len(cases), max_payload=arena.nbytes, semantics=sem)
    codes, fp, img = eng.verify_raw_host(arena, off, sz, want_img=True)
    eng.close()
    np.testing.assert_array_equal(fp, wfp)
    np.testing.assert_array_equal(crcs(fp, img), crcs(wfp, wimg))
    np.testing.assert_array_equal(codes, want)
    assert (codes == 0).sum() > 1000 and (codes == -16).sum() > 100 and (codes == -1).sum() > 50


def test_verify_raw_device_full_size(oracle):
    """1M x 1232-byte raw payloads (BASELINE configs[1]) on the device path; 1 in 97 payloads is
    corrupted (parse failure or bad signature); exactly those are rejected."""
    import torch
    from firedancer_amd import Engine, engine, synth
    n = 1 << 20
    payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, seed=4321)
    off = desc["payload_off"].copy()
    sz = desc["payload_sz"].copy()
    bad = np.arange(0, n, 97)
    sz[bad[0::2]] -= 1                                    # truncated: trailing-bytes check fails -> parse error
    payload[off[bad[1::2]] + 1000] ^= 0x5a                # filler-data byte flip -> ERR_MSG
    raw, lanes = engine.raw_records(payload, off, sz)
    assert lanes == n
    eng = Engine(device=0, max_txn=n, max_sig=n)
    d_pay = torch.from_numpy(payload).cuda()
    d_raw = torch.from_numpy(raw.view(np.uint8)).cuda()
    d_out = torch.empty(n, dtype=torch.int8, device="cuda")
    eng.verify_raw_device(d_pay.data_ptr(), d_raw.data_ptr(), n, lanes, d_out.data_ptr(), None, None,
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    eng.close()
    want = np.zeros(n, np.int8)
    want[bad[0::2]] = engine.FDGPU_ERR_PARSE
    want[bad[1::2]] = -3
    np.testing.assert_array_equal(out, want)


def test_async_raw_submit_poll(oracle):
    """submit_raw / poll_raw: in-order completions, codes and fd_txn_t images match the oracle,
    with several slots in flight and mixed desc / raw submissions."""
    from firedancer_amd import Engine
    cases = _raw_cases()
    arena, off, sz = tb.pack(cases)
    want, wfp, wimg = raw_expect.expected_codes(oracle, arena, off, sz)
    eng = Engine(device=0, max_txn=300, max_sig=300 * 16, max_payload=300 * 1240)
    got_t, got_c, got_fp, got_img = [], [], [], []
    pending = 0
    for i, c in enumerate(cases):
        while True:
            rc = eng.submit_raw(c, 1000 + i)
            if rc != -2:
                break
            t, cd, fp, im = eng.poll_raw(256, blocking=True)
            got_t.append(t); got_c.append(cd); got_fp.append(fp); got_img.append(im)
        assert rc == 0
        if i % 97 == 0:
            t, cd, fp, im = eng.poll_raw(64)
            got_t.append(t); got_c.append(cd); got_fp.append(fp); got_img.append(im)
    eng.flush()
    while sum(len(t) for t in got_t) < len(cases):
        t, cd, fp, im = eng.poll_raw(512, blocking=True)
        got_t.append(t); got_c.append(cd); got_fp.append(fp); got_img.append(im)
    eng.close()
    tags = np.concatenate(got_t); codes = np.concatenate(got_c); fps = np.concatenate(got_fp)
    imgs = np.concatenate(got_img)
    np.testing.assert_array_equal(tags, 1000 + np.arange(len(cases)))
    np.testing.assert_array_equal(codes, want)
    np.testing.assert_array_equal(fps, wfp)
    np.testing.assert_array_equal(crcs(fps, imgs), crcs(wfp, wimg))
