"""Helpers to turn tests/golden fixtures into batch inputs (payload arena + descriptors)."""
import os

import numpy as np

DESC_DTYPE = np.dtype([("payload_off", "<u4"), ("sig_base", "<u4"), ("payload_sz", "<u2"),
                       ("message_off", "<u2"), ("acct_addr_off", "<u2"), ("signature_off", "u1"),
                       ("sig_cnt", "u1")])


def vectors_as_txns(v, idx=None):
    """Each single-signature vector becomes a 1-signer transaction: sig | pub | msg."""
    n_all = len(v["msg_sz"])
    idx = np.arange(n_all) if idx is None else np.asarray(idx)
    arena = bytearray(); desc = []
    for s, i in enumerate(idx):
        m = v["msg_arena"][v["msg_off"][i]: v["msg_off"][i] + v["msg_sz"][i]].tobytes()
        while len(arena) % 4 != (s % 4):
            arena += b"\x5a"
        off = len(arena)
        arena += v["sig"][i].tobytes() + v["pub"][i].tobytes() + m
        desc.append((off, s, 96 + len(m), 96, 64, 0, 1))
    payload = np.frombuffer(bytes(arena) + bytes(256), np.uint8).copy()
    return payload, np.array(desc, dtype=DESC_DTYPE)


def txns_fixture(t):
    desc = t["desc"].reshape(-1).view(DESC_DTYPE).copy()
    return t["payload"].copy(), desc, int(t["sig_total"][0])


def load_vectors():
    return dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vectors.npz")))
