import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    return {k: dict(np.load(os.path.join(d, f"{k}.npz"))) for k in ("vectors", "txns", "sha")}


# Every GPU test runs on both engine paths (include/fd_ed25519_gpu.h,
# fdgpu_ed25519_set_small_batch_max): "throughput" (half-size scalars,
# fd_gpu_lattice.h: R decoded, a 128-doubling walk, Q == O), "throughput_full"
# (half = 0: the 252-doubling walk, R checked after one batched inversion per
# 256 signatures) and "latencyN" (one fused prep, R decoded up front, N = 8,
# 4, 2 or 1 lanes per signature in the DSM; 8 = the half-size walk's terms
# split over two quads; "latency8x" the same with every prep / walk workgroup
# alone on its CU, fdgpu_ed25519_set_cu_exclusive; "latency4s" the 4-lane walk after a prep whose hash role runs
# one lane per signature instead of a quad, fdgpu_debug_opts_t.quad_sha).  The choice goes through the engine's explicit test
# hook, fdgpu_debug_set_opts, which every context created afterwards reads --
# contexts the verify tile library creates too.  The product never reads
# these from the environment.
def pytest_generate_tests(metafunc):
    if metafunc.definition.get_closest_marker("gpu") is not None and "engine_path" in metafunc.fixturenames:
        metafunc.parametrize("engine_path", ["throughput", "throughput_full", "latency8", "latency4", "latency2",
                                            "latency1", "latency8x", "latency4s"],
                            indirect=True)


def engine_opts(path: str, **kw) -> dict:
    """fdgpu_debug_opts_t fields selecting an engine path (see above)."""
    o = dict(small_batch_max=0 if path.startswith("throughput") else 2**63,
             half=0 if path == "throughput_full" else 1,
             dsm_lanes=int(path.rstrip("xs")[-1]) if path.startswith("latency") else 0,
             # "s": the prep's hash role on one lane per signature (the default runs it on a quad up to 8,192)
             quad_sha=-1 if path.endswith("s") else 0,
             # "x": workgroups alone on their CUs (set_cu_exclusive); the other latency paths explicitly off (-1),
             # so verify tiles, whose default is on, run them as named too
             cu_exclusive=1 if path.endswith("x") else (-1 if path.startswith("latency") else 0))
    o.update(kw)
    return o


@pytest.fixture(autouse=True)
def engine_path(request):
    path = getattr(request, "param", None)
    if path is not None:
        from firedancer_amd import engine
        engine.debug_set_opts(**engine_opts(path))
        yield path
        engine.debug_reset_opts()
    else:
        yield path
