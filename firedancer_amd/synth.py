"""Synthetic signed transaction batches (ctypes over libfdsynth.so, host C).

Layouts follow the reference's load generator (fd_benchg.c large_noop_t:
1232-byte single-signer txns, message = bytes 65..1231).  Used by bench.py
and the tests to build batches in the engine's arena + descriptor format.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .engine import DESC_DTYPE, PKG_DIR

LARGE_NOOP = 0   # 1232-byte single-signer txn (BASELINE configs[1])
SMALL_MSG = 1    # single signer, 200-byte message (BASELINE configs[0])
MULTI = 2        # 1..max_signers signers over one <=1232-byte message (configs[3])

_KEY_SZ = 128
_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(PKG_DIR, "libfdsynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(path)
        L.fdsynth_keys.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        L.fdsynth_txns.restype = ctypes.c_size_t
        L.fdsynth_txns.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.c_int]
        _lib = L
    return _lib


def keys(n: int, seed: int = 1234) -> np.ndarray:
    k = np.zeros((n, _KEY_SZ), np.uint8)
    _load().fdsynth_keys(k.ctypes.data, n, seed)
    return k


def pubkey(keys_arr: np.ndarray, i: int) -> bytes:
    return keys_arr[i, 32:64].tobytes()


def make_batch(n: int, kind: int = LARGE_NOOP, max_signers: int = 1, invalid_frac: float = 0.0,
               seed: int = 1234, nkeys: int = 1024, threads: int | None = None, key_arr: np.ndarray | None = None):
    """Returns (payload uint8[], desc DESC_DTYPE[], expect int8[] (intended AVX-512 txn code), sig_total)."""
    stride = 272 if kind == SMALL_MSG else 1232
    payload = np.zeros(n * stride + 1024, np.uint8)
    desc = np.zeros(n, DESC_DTYPE)
    expect = np.zeros(n, np.int8)
    if key_arr is None:
        key_arr = keys(nkeys, seed ^ 0x5eed)
    threads = threads or min(16, os.cpu_count() or 1)
    nsig = _load().fdsynth_txns(payload.ctypes.data, stride, desc.ctypes.data, expect.ctypes.data, n, kind,
                                max_signers, float(invalid_frac), seed, key_arr.ctypes.data, len(key_arr), threads)
    return payload, desc, expect, int(nsig)
