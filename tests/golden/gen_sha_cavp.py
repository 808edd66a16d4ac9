#!/usr/bin/env python3
"""Extract the NIST CAVP SHA-512 ShortMsg / LongMsg vectors the reference
tests with (src/ballet/sha512/cavp/SHA512{Short,Long}Msg.rsp, used by
test_sha512.c:5-6,167-169) into tests/golden/sha_cavp.npz (data only).
Run in the build container only."""
import os

import numpy as np

CAVP = "/root/reference/src/ballet/sha512/cavp"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse(path):
    out, ln, msg = [], None, None
    for line in open(path):
        line = line.strip()
        if line.startswith("Len ="):
            ln = int(line.split("=")[1])
        elif line.startswith("Msg ="):
            msg = bytes.fromhex(line.split("=")[1].strip())
        elif line.startswith("MD =") and ln is not None:
            out.append((msg[: ln // 8], bytes.fromhex(line.split("=")[1].strip())))
            ln = None
    return out


def main():
    vecs = parse(os.path.join(CAVP, "SHA512ShortMsg.rsp")) + parse(os.path.join(CAVP, "SHA512LongMsg.rsp"))
    lens = np.array([len(m) for m, _ in vecs], np.uint32)
    data = np.frombuffer(b"".join(m for m, _ in vecs), np.uint8)
    md = np.frombuffer(b"".join(d for _, d in vecs), np.uint8).reshape(-1, 64)
    np.savez_compressed(os.path.join(HERE, "sha_cavp.npz"), data=data, lens=lens, md=md)
    print(len(vecs), "vectors,", data.nbytes, "message bytes")


if __name__ == "__main__":
    main()
