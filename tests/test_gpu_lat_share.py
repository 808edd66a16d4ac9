"""fdgpu_ed25519_set_lat_share: with cu_exclusive on, the latency path's walk keeps within the context's
share of the CUs by taking fewer lanes per signature (include/fd_ed25519_gpu.h).  The verify tile gives each
of its n contexts 1/n (fd_verify_gpu.c vt_ctx_new), so two staggered batches' exclusive walks never need
more CUs than the device has.  Checked: the lanes each batch size and share gets (fdgpu_ed25519_front_batch),
and that every path's codes are the generator's intended ones (the engine paths themselves are pinned
against the oracle and the reference in test_gpu_parity.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NCU = 256      # MI355X; the expectations below assume no CUs reserved for gathers


@pytest.mark.parametrize("n,share,lanes", [(3000, 2, 8), (5000, 2, 4), (5000, 0, 8), (9000, 2, 2), (9000, 4, 1),
                                           (20000, 2, 1), (20000, 0, 2)])
def test_lat_share_lanes(n, share, lanes, engine_path):
    import torch
    from firedancer_amd import Engine, engine, synth
    if engine_path != "throughput":
        pytest.skip("sets its own path: runs once")
    engine.debug_reset_opts()                          # the product's defaults (no forced lanes)
    if torch.cuda.get_device_properties(0).multi_processor_count != NCU:
        pytest.skip("expectations assume 256 CUs")
    payload, desc, expect, nsig = synth.make_batch(n, synth.LARGE_NOOP, 1, 0.1, seed=77 + n)
    eng = Engine(device=0, max_txn=n, max_sig=nsig, max_payload=n * 1240)
    try:
        eng.set_small_batch_max(2**64 - 1)            # every batch on the latency path
        eng.set_cu_exclusive(1)
        eng.set_lat_share(share)
        for i in range(n):
            o, z = int(desc["payload_off"][i]), int(desc["payload_sz"][i])
            assert eng.submit_raw(payload[o:o + z].tobytes(), i) == 0
        eng.flush()
        fb = eng.front_batch()
        assert fb is not None and fb[0] == n
        assert fb[2] == lanes
        tags, codes = [], []
        while sum(len(t) for t in tags) < n:
            t, c, _, _ = eng.poll_raw(n, blocking=True)
            tags.append(t)
            codes.append(c)
        np.testing.assert_array_equal(np.concatenate(tags), np.arange(n))
        np.testing.assert_array_equal(np.concatenate(codes), expect)
    finally:
        eng.close()
