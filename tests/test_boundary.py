"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what
include/*.h declares (no compute calls -- no GPU here)."""
import os
import re
import subprocess

from firedancer_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions(name="fd_ed25519_gpu.h"):
    txt = open(os.path.join(ROOT, "include", name)).read()
    if name != "fd_ed25519_gpu.h":
        txt = txt.split('#include "fd_ed25519_gpu.h"', 1)[1]
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"static inline[^{]*\{.*?\n\}", "", txt, flags=re.S)    # header-only helpers, not exports
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)) - {"sizeof"})


def test_header_matches_exports_list():
    assert sorted(engine.EXPORTS) == _header_functions()


def test_vtile_header_matches_exports_list():
    from firedancer_amd import vtile
    assert sorted(vtile.EXPORTS) == _header_functions("fd_verify_gpu.h")


def test_vtile_library_exports():
    from firedancer_amd import vtile
    out = subprocess.run(["nm", "-D", "--defined-only", vtile.LIB_PATH], capture_output=True, text=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert [n for n in vtile.EXPORTS if n not in syms] == []


def test_library_loads_and_exports():
    lib = engine.load_library()
    for name in engine.EXPORTS:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True, text=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for name in engine.EXPORTS:
        assert name in syms, name


def test_library_has_gfx950_code_object():
    data = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_strerror_no_gpu_needed():
    lib = engine.load_library()
    assert lib.fd_ed25519_strerror(0) == b"success"
    assert lib.fd_ed25519_strerror(-1) == b"bad signature"
    assert lib.fd_ed25519_strerror(-2) == b"bad public key"
    assert lib.fd_ed25519_strerror(-3) == b"bad message"
    assert lib.fd_ed25519_strerror(7) == b"unknown"


def test_desc_layout():
    import numpy as np
    assert engine.DESC_DTYPE.itemsize == 16
    assert [engine.DESC_DTYPE.fields[k][1] for k in engine.DESC_DTYPE.names] == [0, 4, 8, 10, 12, 14, 15]
    assert np.dtype(engine.DESC_DTYPE).names[-1] == "sig_cnt"


def test_ctx_new_rejects_bad_sizes_without_gpu():
    lib = engine.load_library()
    assert not lib.fdgpu_ed25519_ctx_new(0, 0, 16, 0, 0)
    assert engine.last_error() == "bad sizes"
    assert not lib.fdgpu_ed25519_ctx_new(0, 16, 16, 0, 7)
    assert engine.last_error() == "bad semantics"


def test_raw_record_layout_and_staging():
    import numpy as np
    assert engine.RAW_DTYPE.itemsize == 16
    assert [engine.RAW_DTYPE.fields[k][1] for k in engine.RAW_DTYPE.names] == [0, 4, 8, 10, 11]
    # sig lanes = first payload byte when in 1..16 (fd_txn_parse.c:86), else 0; sig_base = prefix
    payload = np.array([1, 0, 0, 3, 0, 0, 17, 0, 0, 0, 0, 0, 2, 0], np.uint8)
    off = np.array([0, 3, 6, 9, 12], np.uint32)
    sz = np.array([3, 3, 3, 0, 2], np.uint16)
    raw, lanes = engine.raw_records(payload, off, sz)
    assert raw["sig_lanes"].tolist() == [1, 3, 0, 0, 2] and raw["sig_base"].tolist() == [0, 1, 4, 4, 4] and lanes == 6


REF_SRC = "/root/reference/src"


def _compile_dropin(inc_dir):
    return subprocess.run(["gcc", "-std=gnu17", "-Wall", "-Wextra", "-Werror", "-c", "-o", os.devnull,
                           f"-I{REF_SRC}", f"-I{inc_dir}", os.path.join(ROOT, "tests", "boundary", "dropin_with_ref_header.c")],
                          capture_output=True, text=True)


def test_dropin_prototypes_compile_beside_the_reference_header(tmp_path):
    """the reference's src/ballet/ed25519/fd_ed25519.h, included in place, and then
    include/fd_ed25519_gpu.h in one translation unit under -Wall -Werror, calling both drop-ins -- and, as a
    control, the same with a copy of our header whose fd_ed25519_verify takes a 32-bit msg_sz, which must not
    compile (so the check bites).  Needs the reference tree (this container; absent on the GPU box)."""
    import pytest
    import shutil
    if not os.path.exists(os.path.join(REF_SRC, "ballet", "ed25519", "fd_ed25519.h")):
        pytest.skip("reference tree absent")
    r = _compile_dropin(os.path.join(ROOT, "include"))
    assert r.returncode == 0, r.stderr[-2000:]
    bad = tmp_path / "inc"
    bad.mkdir()
    src = open(os.path.join(ROOT, "include", "fd_ed25519_gpu.h")).read()
    mut = src.replace("fd_ed25519_verify( unsigned char const   msg[], /* msg_sz */\n                   unsigned long  ",
                      "fd_ed25519_verify( unsigned char const   msg[], /* msg_sz */\n                   unsigned int   ", 1)
    assert mut != src
    (bad / "fd_ed25519_gpu.h").write_text(mut)
    assert _compile_dropin(str(bad)).returncode != 0
